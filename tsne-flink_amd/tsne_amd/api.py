"""Host-side operators mirroring TsneHelpers (TsneHelpers.scala), over the C ABI.

Arguments are numpy arrays (host) or torch CUDA tensors (device API).  Names
and argument meaning follow the reference's Scala methods.
"""
import ctypes as C

import numpy as np

from ._lib import METRICS, UNIQUE_ID_BYTES, CommOps, Params, check, lib


def _ptr(a):
    if a is None:
        return None
    if hasattr(a, "data_ptr"):       # torch tensor (device API)
        return C.c_void_p(a.data_ptr())
    return C.c_void_p(a.ctypes.data)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _csr(row_ptr, col, P, n):
    """CSR arrays in the ABI's types.  The caller must keep the returned arrays
    referenced until the library call returns: a converted temporary passed
    straight into _ptr() would be freed before the library reads it."""
    rp = np.ascontiguousarray(row_ptr, dtype=np.int64)
    cl = np.ascontiguousarray(col, dtype=np.int32)
    pv = np.ascontiguousarray(P, dtype=np.float64)
    if rp.shape != (n + 1,):
        raise ValueError("row_ptr has shape %s, expected (%d,)" % (rp.shape, n + 1))
    if cl.shape != (int(rp[-1]),) or pv.shape != cl.shape:
        raise ValueError("col / P must hold row_ptr[n] = %d entries" % int(rp[-1]))
    return rp, cl, pv


def _inout(n, c, **arrays):
    """Arrays the library writes in place must already be float64, C-contiguous, n x c."""
    for name, a in arrays.items():
        if not (isinstance(a, np.ndarray) and a.dtype == np.float64 and a.flags.c_contiguous
                and a.shape == (n, c)):
            raise ValueError("%s must be a C-contiguous float64 array of shape (%d, %d)" % (name, n, c))


def default_params(**kw):
    p = Params()
    lib().tsne_params_default(C.byref(p))
    for k, v in kw.items():
        if k == "metric" and isinstance(v, str):
            v = METRICS[v]
        setattr(p, k, v)
    return p


class Context:
    """One tsne_ctx (one GPU, optionally one rank of an RCCL communicator)."""

    def __init__(self, device=0):
        self._h = C.c_void_p()
        check(lib().tsne_ctx_create(device, C.byref(self._h)))

    @classmethod
    def multi(cls, devices):
        """tsne_ctx_create_multi: one handle over several ranks (distinct GPUs over
        RCCL, or the same GPU repeated = in-process loopback ranks)."""
        self = cls.__new__(cls)
        self._h = C.c_void_p()
        devs = np.ascontiguousarray(devices, dtype=np.int32)
        check(lib().tsne_ctx_create_multi(_ptr(devs), len(devs), C.byref(self._h)))
        return self

    def set_option(self, key, value):
        """tsne_ctx_set_option: a per-handle tunable (include/tsne_hip.h lists the keys)."""
        check(lib().tsne_ctx_set_option(self._h, key.encode(), float(value)))

    def get_option(self, key):
        out = C.c_double()
        check(lib().tsne_ctx_get_option(self._h, key.encode(), C.byref(out)))
        return out.value

    def counter(self, name):
        """tsne_ctx_counter: a diagnostic counter of the last call (e.g. "bh.narrow_groups")."""
        out = C.c_int64()
        check(lib().tsne_ctx_counter(self._h, name.encode(), C.byref(out)))
        return out.value

    def loop_profile(self):
        """tsne_ctx_loop_profile: the loopback group's serial-mode summary (dict;
        option loop_serial), or None."""
        import json
        n = C.c_int64()
        check(lib().tsne_ctx_loop_profile(self._h, None, 0, C.byref(n)))
        if n.value == 0:
            return None
        buf = C.create_string_buffer(n.value + 1)
        check(lib().tsne_ctx_loop_profile(self._h, buf, n.value + 1, C.byref(n)))
        return json.loads(buf.value.decode())

    def rank_world(self):
        r, w = C.c_int32(), C.c_int32()
        check(lib().tsne_ctx_rank(self._h, C.byref(r), C.byref(w)))
        return r.value, w.value

    def close(self):
        if self._h:
            lib().tsne_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # ---- multi-GPU
    @staticmethod
    def unique_id():
        buf = C.create_string_buffer(UNIQUE_ID_BYTES)
        check(lib().tsne_comm_unique_id(buf))
        return buf.raw

    def init_comm(self, rank, world, uid):
        check(lib().tsne_ctx_init_comm(self._h, rank, world, uid))

    def init_comm_callbacks(self, rank, world, allreduce_sum, allgatherv):
        """tsne_ctx_init_comm_callbacks: the library's collectives carried by the
        caller.  allreduce_sum(ndarray) sums a float64 / uint64 array over the ranks
        in place; allgatherv(ndarray_u8, offsets) makes rank r's bytes
        [off[r], off[r+1]) reach every rank, in place."""
        def f64(_, buf, count):
            try:
                allreduce_sum(np.ctypeslib.as_array(buf, shape=(count,)))
                return 0
            except Exception:   # noqa: BLE001 -- reported to the library as a failed collective
                return 1

        def u64(_, buf, count):
            try:
                allreduce_sum(np.ctypeslib.as_array(buf, shape=(count,)))
                return 0
            except Exception:   # noqa: BLE001
                return 1

        def agv(_, buf, off):
            try:
                o = np.ctypeslib.as_array(off, shape=(world + 1,)).copy()
                allgatherv(np.ctypeslib.as_array(C.cast(buf, C.POINTER(C.c_uint8)), shape=(int(o[-1]),)), o)
                return 0
            except Exception:   # noqa: BLE001
                return 1
        ops = CommOps()
        ops.allreduce_sum_f64 = CommOps._fields_[0][1](f64)
        ops.allreduce_sum_u64 = CommOps._fields_[1][1](u64)
        ops.allgatherv = CommOps._fields_[2][1](agv)
        self._comm_ops = ops   # the callbacks must outlive the context's use of them
        check(lib().tsne_ctx_init_comm_callbacks(self._h, rank, world, C.byref(ops), None))

    def set_stream(self, stream_ptr):
        check(lib().tsne_ctx_set_stream(self._h, C.c_void_p(stream_ptr) if stream_ptr else None))
        self._stream_ptr = int(stream_ptr or 0)

    def _fence(self, t):
        """The dev_* operators read torch tensors on the context's stream: unless
        that is torch's current stream (set_stream), wait for torch's current
        stream first, so inputs torch just produced are complete (the context's
        own stream is non-blocking; the null stream cannot be shared).  Outputs
        are ready after synchronize()."""
        import torch
        s = torch.cuda.current_stream(t.device)
        if not getattr(self, "_stream_ptr", 0) or s.cuda_stream != self._stream_ptr:
            s.synchronize()

    def synchronize(self):
        check(lib().tsne_ctx_synchronize(self._h))

    def debug_wave_log(self):
        """(start, end, kind) per BH wave of the last counting call (options
        wave_log + rep_stats), 100 MHz ticks; kind 0 traversal, 1 narrow, 2 tile."""
        import numpy as np
        n = C.c_int64()
        check(lib().tsne_debug_wave_log(self._h, None, C.c_int64(0), C.byref(n)))
        buf = np.zeros(2 * max(1, n.value), dtype=np.uint64)
        check(lib().tsne_debug_wave_log(self._h, buf.ctypes.data_as(C.c_void_p), C.c_int64(n.value), C.byref(n)))
        buf = buf[:2 * n.value].reshape(-1, 2)
        return buf[:, 0], buf[:, 1] >> np.uint64(2), (buf[:, 1] & np.uint64(3)).astype(np.int32)

    # ---- host operators (TsneHelpers names)
    def kNearestNeighbors(self, X, k, metric="sqeuclidean", q0=0, q1=None):
        """TsneHelpers.scala:41-59 -> (idx[nq, kk] int32, dist[nq, kk] f64)."""
        X = _f64(X)
        n, d = X.shape
        q1 = n if q1 is None else q1
        kk = min(k, n - 1)
        idx = np.zeros((q1 - q0, kk), dtype=np.int32)
        dist = np.zeros((q1 - q0, kk), dtype=np.float64)
        check(lib().tsne_knn(self._h, _ptr(X), n, d, METRICS[metric], k, q0, q1, _ptr(idx), _ptr(dist)))
        return idx, dist

    def pairwiseAffinities(self, row_ptr, dist, perplexity):
        """TsneHelpers.scala:162-180 on CSR rows of distances."""
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
        dist = _f64(dist).ravel()
        p = np.zeros_like(dist)
        check(lib().tsne_pairwise_affinities(self._h, _ptr(row_ptr), _ptr(dist), len(row_ptr) - 1,
                                             perplexity, _ptr(p)))
        return p

    def jointDistribution(self, row_ptr, col, p, n):
        """TsneHelpers.scala:182-196 -> symmetric CSR (rows sorted by column)."""
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
        col = np.ascontiguousarray(col, dtype=np.int32)
        p = _f64(p)
        cap = 2 * len(col) + 1
        orp = np.zeros(n + 1, dtype=np.int64)
        oc = np.zeros(cap, dtype=np.int32)
        ov = np.zeros(cap, dtype=np.float64)
        nnz = C.c_int64()
        check(lib().tsne_joint_distribution(self._h, _ptr(row_ptr), _ptr(col), _ptr(p), n, cap,
                                            _ptr(orp), _ptr(oc), _ptr(ov), C.byref(nnz)))
        return orp, oc[:nnz.value].copy(), ov[:nnz.value].copy()

    def projectKnn(self, X, k, metric="sqeuclidean", iterations=3, shifts=None, seed=0):
        """TsneHelpers.scala:93-160 (--knnMethod project) -> (idx, dist), n x min(k, n-1).
        shifts: (iterations-1) x d uniform [0,1) vectors (default: project_shifts(seed))."""
        X = _f64(X)
        n, d = X.shape
        if shifts is None:
            shifts = project_shifts(iterations, d, seed)
        shifts = _f64(np.asarray(shifts).reshape(max(iterations - 1, 0), d))
        kk = min(k, n - 1)
        idx = np.zeros((n, kk), dtype=np.int32)
        dist = np.zeros((n, kk))
        check(lib().tsne_project_knn(self._h, _ptr(X), n, d, METRICS[metric], k, iterations,
                                     _ptr(shifts) if iterations > 1 else None, _ptr(idx), _ptr(dist)))
        return idx, dist

    def gradient(self, row_ptr, col, P, Y, theta, metric="sqeuclidean", exaggeration=1.0,
                 want_loss=False):
        """TsneHelpers.scala:221-318 -> (grad[n,c], Z, loss or None); c = Y.shape[1]
        is 2 (quadtree) or 3 (the octree extension, tsne_gradient_c)."""
        Y = _f64(Y)
        n, c = Y.shape
        rp, cl, pv = _csr(row_ptr, col, P, n)   # converted copies stay referenced across the call
        grad = np.zeros((n, c))
        z = C.c_double()
        loss = C.c_double()
        check(lib().tsne_gradient_c(self._h, _ptr(rp), _ptr(cl), _ptr(pv), n, c,
                                    _ptr(Y), METRICS[metric], theta, exaggeration, _ptr(grad),
                                    C.byref(z), C.byref(loss) if want_loss else None))
        return grad, z.value, (loss.value if want_loss else None)

    def repulsion(self, Y, theta):
        """QuadTree.computeRepulsiveForce (QuadTree.scala:123-152) for every point
        -> (F[n, c], z[n]); c = Y.shape[1] is 2 or 3 (octree extension)."""
        Y = _f64(Y)
        n, c = Y.shape
        F = np.zeros((n, c))
        z = np.zeros(n)
        check(lib().tsne_repulsion(self._h, _ptr(Y), n, c, theta, _ptr(F), _ptr(z)))
        return F, z

    def dev_repulsion(self, dY, theta, dF, dz):
        self._fence(dY)
        n, c = dY.shape
        check(lib().tsne_dev_repulsion(self._h, _ptr(dY), n, c, theta, _ptr(dF), _ptr(dz)))

    def updateEmbedding(self, grad, Y, upd, gains, min_gain, momentum, learning_rate):
        """TsneHelpers.scala:341-369, in place on Y / upd / gains."""
        n, c = Y.shape
        _inout(n, c, Y=Y, upd=upd, gains=gains)
        g = _f64(grad)
        if g.shape != (n, c):
            raise ValueError("grad has shape %s, expected %s" % (g.shape, (n, c)))
        check(lib().tsne_update_embedding(self._h, n, c, _ptr(g), _ptr(Y), _ptr(upd), _ptr(gains),
                                          min_gain, momentum, learning_rate))

    def centerEmbedding(self, Y):
        """TsneHelpers.scala:320-329, in place."""
        n, c = Y.shape
        _inout(n, c, Y=Y)
        check(lib().tsne_center_embedding(self._h, n, c, _ptr(Y)))

    def initWorkingSet(self, n, n_components=2, seed=0):
        """TsneHelpers.scala:198-219 (seeded) -> (Y, upd, gains)."""
        Y = np.zeros((n, n_components))
        upd = np.zeros_like(Y)
        gains = np.zeros_like(Y)
        check(lib().tsne_init_working_set(self._h, n, n_components, seed, _ptr(Y), _ptr(upd), _ptr(gains)))
        return Y, upd, gains

    def optimize(self, row_ptr, col, P, Y, upd, gains, params):
        """TsneHelpers.scala:396-430, in place; returns {iteration: loss}."""
        n = Y.shape[0]
        if Y.shape[1] != params.n_components:
            raise ValueError("Y has %d columns, params.n_components is %d" % (Y.shape[1], params.n_components))
        _inout(n, params.n_components, Y=Y, upd=upd, gains=gains)   # written in place by the library
        rp, cl, pv = _csr(row_ptr, col, P, n)   # converted copies stay referenced across the call
        cap = params.iterations // 10 + 1
        keys = np.zeros(cap, dtype=np.int32)
        vals = np.zeros(cap)
        nl = C.c_int32()
        check(lib().tsne_optimize(self._h, C.byref(params), _ptr(rp), _ptr(cl), _ptr(pv), n, _ptr(Y),
                                  _ptr(upd), _ptr(gains), _ptr(keys), _ptr(vals), cap, C.byref(nl)))
        return dict(zip(keys[:nl.value].tolist(), vals[:nl.value].tolist()))

    # ---- device operators (torch CUDA tensors)
    def dev_knn(self, dX, k, metric, q0, q1, d_idx, d_dist):
        self._fence(dX)
        n, d = dX.shape
        check(lib().tsne_dev_knn(self._h, _ptr(dX), n, d, METRICS[metric], k, q0, q1, _ptr(d_idx), _ptr(d_dist)))

    def dev_affinities(self, d_row_ptr, d_dist, nrows, perplexity, d_p):
        self._fence(d_dist)
        check(lib().tsne_dev_pairwise_affinities(self._h, _ptr(d_row_ptr), _ptr(d_dist), nrows, perplexity, _ptr(d_p)))

    def dev_joint(self, d_row_ptr, d_col, d_p, n, cap, d_orp, d_oc, d_ov):
        self._fence(d_p)
        nnz = C.c_int64()
        check(lib().tsne_dev_joint_distribution(self._h, _ptr(d_row_ptr), _ptr(d_col), _ptr(d_p), n, cap,
                                                _ptr(d_orp), _ptr(d_oc), _ptr(d_ov), C.byref(nnz)))
        return nnz.value

    def dev_opt_setup(self, params, d_row_ptr, d_col, d_P, n, dY, dupd, dgains):
        self._fence(dY)
        check(lib().tsne_dev_opt_setup(self._h, C.byref(params), _ptr(d_row_ptr), _ptr(d_col), _ptr(d_P), n,
                                       _ptr(dY), _ptr(dupd), _ptr(dgains)))

    def dev_opt_step(self, t):
        check(lib().tsne_dev_opt_step(self._h, t))

    def dev_opt_sync(self):
        check(lib().tsne_dev_opt_sync(self._h))

    def dev_opt_last_z(self):
        """Z of the last tsne_dev_opt_step (the normaliser its gradient and loss used)."""
        z = C.c_double()
        check(lib().tsne_dev_opt_last_z(self._h, C.byref(z)))
        return z.value

    def dev_opt_losses(self, cap=1024):
        keys = np.zeros(cap, dtype=np.int32)
        vals = np.zeros(cap)
        nl = C.c_int32()
        check(lib().tsne_dev_opt_losses(self._h, _ptr(keys), _ptr(vals), cap, C.byref(nl)))
        k = min(nl.value, cap)
        return dict(zip(keys[:k].tolist(), vals[:k].tolist()))

    def dev_balance_cuts(self, bcost, n, world, bounds):
        """tsne_dev_balance_cuts on device tensors (uint64/int64 bucket costs, int64 bounds[world+1])."""
        self._fence(bcost)
        check(lib().tsne_dev_balance_cuts(self._h, _ptr(bcost), n, world, _ptr(bounds)))

    def dev_opt_attract_log(self):
        """-> list of (iteration, standalone, ms) for every attraction launch since setup."""
        cnt = C.c_int32()
        check(lib().tsne_dev_opt_attract_log(self._h, None, None, None, 0, C.byref(cnt)))
        k = cnt.value
        it = np.zeros(max(k, 1), dtype=np.int32)
        sa = np.zeros(max(k, 1), dtype=np.int32)
        ms = np.zeros(max(k, 1))
        check(lib().tsne_dev_opt_attract_log(self._h, _ptr(it), _ptr(sa), _ptr(ms), k, C.byref(cnt)))
        return [(int(it[e]), int(sa[e]), float(ms[e])) for e in range(k)]

    def stage_ms(self, stage):
        """Per-interval kernel times (ms) of a stage timer (tsne_ctx_stage_ms)."""
        cnt = C.c_int32()
        check(lib().tsne_ctx_stage_ms(self._h, stage.encode(), None, 0, C.byref(cnt)))
        out = np.zeros(max(cnt.value, 1))
        check(lib().tsne_ctx_stage_ms(self._h, stage.encode(), _ptr(out), cnt.value, C.byref(cnt)))
        return out[:cnt.value].tolist()

    def dev_opt_profile(self, enable=-1):
        """-> (stage ms[5], BH counters [visits, moment evaluations, dense pair terms,
        wave-level pops, wave-level dense tile points, lane child evaluations, wave child slots, heaviest wave, max wave pops,
        max wave dense points])"""
        ms = np.zeros(5)
        cnt = np.zeros(10, dtype=np.int64)
        check(lib().tsne_dev_opt_profile(self._h, enable, _ptr(ms), _ptr(cnt)))
        return ms, cnt.tolist()


def project_shifts(iterations, d, seed=0):
    """The projectKnn shift vectors: iterations-1 rows of uniform [0,1)^d
    (DenseVector.rand, TsneHelpers.scala:97; seeded here, the reference is not)."""
    return np.random.default_rng(seed).random((max(iterations - 1, 0), d))
