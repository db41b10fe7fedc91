"""ctypes bindings to oracle/liboracle.so -- the CPU fp64 restatement.

Test infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module.
"""
import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
ORACLE_DIR = ROOT / "oracle"
METRICS = {"sqeuclidean": 0, "euclidean": 1, "cosine": 2}

_lib = None


def lib():
    global _lib
    if _lib is None:
        so = ORACLE_DIR / "liboracle.so"
        if not so.exists():
            subprocess.check_call(["make", "-s", "-C", str(ORACLE_DIR)])
        _lib = C.CDLL(str(so))
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t)) if a is not None else None


D = C.c_double
I32 = C.c_int32
I64 = C.c_int64


def knn(X, k, metric="sqeuclidean", q0=0, q1=None, threads=1):
    X = np.ascontiguousarray(X, dtype=np.float64)
    n, d = X.shape
    q1 = n if q1 is None else q1
    kk = min(k, n - 1)
    idx = np.zeros((q1 - q0, kk), dtype=np.int32)
    dist = np.zeros((q1 - q0, kk), dtype=np.float64)
    rc = lib().oracle_knn(_p(X, D), I64(n), I32(d), C.c_int(METRICS[metric]), I32(k),
                          I64(q0), I64(q1), _p(idx, I32), _p(dist, D), C.c_int(threads))
    assert rc == 0, rc
    return idx, dist


def affinities(row_ptr, dist, perplexity):
    row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
    dist = np.ascontiguousarray(dist, dtype=np.float64).ravel()
    p = np.zeros_like(dist)
    iters = np.zeros(len(row_ptr) - 1, dtype=np.int32)
    rc = lib().oracle_affinities(_p(row_ptr, I64), _p(dist, D), I64(len(row_ptr) - 1),
                                 D(perplexity), _p(p, D), _p(iters, I32))
    assert rc == 0
    return p, iters


def joint(row_ptr, col, p, n):
    row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
    col = np.ascontiguousarray(col, dtype=np.int32)
    p = np.ascontiguousarray(p, dtype=np.float64)
    cap = 2 * len(col) + 1
    orp = np.zeros(n + 1, dtype=np.int64)
    oc = np.zeros(cap, dtype=np.int32)
    ov = np.zeros(cap, dtype=np.float64)
    nnz = I64(0)
    rc = lib().oracle_joint(_p(row_ptr, I64), _p(col, I32), _p(p, D), I64(n), _p(orp, I64),
                            _p(oc, I32), _p(ov, D), I64(cap), C.byref(nnz))
    assert rc == 0, rc
    return orp, oc[:nnz.value].copy(), ov[:nnz.value].copy()


def gradient(row_ptr, col, val, Y, theta, metric="sqeuclidean", exaggeration=1.0,
             want_loss=False, threads=1):
    n = Y.shape[0]
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    grad = np.zeros((n, 2))
    rep = np.zeros((n, 2))
    attr = np.zeros((n, 2))
    zi = np.zeros(n)
    visits = np.zeros(n, dtype=np.int64)
    z = D(0)
    loss = D(0)
    rc = lib().oracle_gradient(_p(np.ascontiguousarray(row_ptr, np.int64), I64),
                               _p(np.ascontiguousarray(col, np.int32), I32),
                               _p(np.ascontiguousarray(val, np.float64), D), I64(n), _p(Y, D),
                               C.c_int(METRICS[metric]), D(theta), D(exaggeration),
                               _p(grad, D), C.byref(z), C.byref(loss) if want_loss else None,
                               _p(rep, D), _p(zi, D), _p(attr, D), _p(visits, I64),
                               C.c_int(threads))
    assert rc == 0
    return dict(grad=grad, Z=z.value, loss=loss.value if want_loss else None, rep=rep,
                zi=zi, attr=attr, visits=visits)


def repulsion(Y, theta, q0=0, q1=None, threads=1):
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    n = Y.shape[0]
    q1 = n if q1 is None else q1
    rep = np.zeros((q1 - q0, 2))
    zi = np.zeros(q1 - q0)
    rc = lib().oracle_repulsion(_p(Y, D), I64(n), D(theta), I64(q0), I64(q1), _p(rep, D),
                                _p(zi, D), C.c_int(threads))
    assert rc == 0
    return rep, zi


def update(grad, Y, upd, gains, min_gain, momentum, lr):
    n, c = Y.shape
    for a in (grad, Y, upd, gains):
        assert a.dtype == np.float64 and a.flags.c_contiguous
    lib().oracle_update(I64(n), I32(c), _p(grad, D), _p(Y, D), _p(upd, D), _p(gains, D),
                        D(min_gain), D(momentum), D(lr))


def center(Y):
    n, c = Y.shape
    lib().oracle_center(I64(n), I32(c), _p(Y, D))


def optimize(row_ptr, col, val, Y, upd, gains, metric="sqeuclidean", learning_rate=1000.0,
             iterations=300, early_exaggeration=4.0, initial_momentum=0.5,
             final_momentum=0.8, theta=0.25, threads=1):
    n = Y.shape[0]
    keys = np.zeros(iterations // 10 + 1, dtype=np.int32)
    vals = np.zeros(iterations // 10 + 1)
    nl = I32(0)
    rc = lib().oracle_optimize(_p(np.ascontiguousarray(row_ptr, np.int64), I64),
                               _p(np.ascontiguousarray(col, np.int32), I32),
                               _p(np.ascontiguousarray(val, np.float64), D), I64(n),
                               _p(Y, D), _p(upd, D), _p(gains, D), C.c_int(METRICS[metric]),
                               D(learning_rate), I32(iterations), D(early_exaggeration),
                               D(initial_momentum), D(final_momentum), D(theta),
                               _p(keys, I32), _p(vals, D), C.byref(nl), C.c_int(threads))
    assert rc == 0
    return dict(zip(keys[:nl.value].tolist(), vals[:nl.value].tolist()))


def repulsion_queries(Y, theta, Q, threads=1):
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    Q = np.ascontiguousarray(Q, dtype=np.float64)
    rep = np.zeros((Q.shape[0], 2))
    zi = np.zeros(Q.shape[0])
    rc = lib().oracle_repulsion_queries(_p(Y, D), I64(Y.shape[0]), D(theta), _p(Q, D), I64(Q.shape[0]),
                                        _p(rep, D), _p(zi, D), C.c_int(threads))
    assert rc == 0
    return rep, zi


class Tree:
    """The reference quadtree of all points of Y (oracle_tree_build), kept for
    several query batches: the CPU baseline times the build and the queries
    apart."""

    def __init__(self, Y):
        self.Y = np.ascontiguousarray(Y, dtype=np.float64)
        L = lib()
        L.oracle_tree_build.restype = C.c_void_p
        L.oracle_tree_build.argtypes = [C.POINTER(D), I64]
        L.oracle_tree_free.argtypes = [C.c_void_p]
        L.oracle_tree_query.argtypes = [C.c_void_p, D, C.POINTER(D), I64, C.POINTER(D), C.POINTER(D),
                                        C.POINTER(I64), C.c_int]
        self.h = L.oracle_tree_build(_p(self.Y, D), I64(self.Y.shape[0]))
        assert self.h

    def query(self, theta, Q, threads=1):
        Q = np.ascontiguousarray(Q, dtype=np.float64)
        rep = np.zeros((Q.shape[0], 2))
        zi = np.zeros(Q.shape[0])
        v = I64(0)
        rc = lib().oracle_tree_query(self.h, D(theta), _p(Q, D), I64(Q.shape[0]), _p(rep, D), _p(zi, D),
                                     C.byref(v), C.c_int(threads))
        assert rc == 0
        return rep, zi, v.value

    def close(self):
        if self.h:
            lib().oracle_tree_free(self.h)
            self.h = None

    def __del__(self):
        self.close()


def attraction_rows(row_ptr, col, val, Y, rep, Z, r0, r1, metric="sqeuclidean", exaggeration=1.0,
                    want_loss=False):
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    rep = np.ascontiguousarray(rep, dtype=np.float64)
    grad = np.zeros((r1 - r0, 2))
    loss = D(0)
    rc = lib().oracle_attraction_rows(_p(np.ascontiguousarray(row_ptr, np.int64), I64),
                                      _p(np.ascontiguousarray(col, np.int32), I32),
                                      _p(np.ascontiguousarray(val, np.float64), D), I64(Y.shape[0]),
                                      _p(Y, D), C.c_int(METRICS[metric]), D(exaggeration), _p(rep, D),
                                      D(Z), I64(r0), I64(r1), _p(grad, D),
                                      C.byref(loss) if want_loss else None)
    assert rc == 0
    return grad, (loss.value if want_loss else None)


def gradient3(row_ptr, col, val, Y, theta, metric="sqeuclidean", exaggeration=1.0,
              want_loss=False, threads=1):
    """3-D extension (octree restatement, parity unpinned: see tsne_oracle.h)."""
    n = Y.shape[0]
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    grad = np.zeros((n, 3))
    rep = np.zeros((n, 3))
    zi = np.zeros(n)
    z = D(0)
    loss = D(0)
    rc = lib().oracle_gradient3(_p(np.ascontiguousarray(row_ptr, np.int64), I64),
                                _p(np.ascontiguousarray(col, np.int32), I32),
                                _p(np.ascontiguousarray(val, np.float64), D), I64(n), _p(Y, D),
                                C.c_int(METRICS[metric]), D(theta), D(exaggeration),
                                _p(grad, D), C.byref(z), C.byref(loss) if want_loss else None,
                                _p(rep, D), _p(zi, D), C.c_int(threads))
    assert rc == 0
    return dict(grad=grad, Z=z.value, loss=loss.value if want_loss else None, rep=rep, zi=zi)


def optimize3(row_ptr, col, val, Y, upd, gains, metric="sqeuclidean", learning_rate=1000.0,
              iterations=300, early_exaggeration=4.0, initial_momentum=0.5,
              final_momentum=0.8, theta=0.25, threads=1):
    n = Y.shape[0]
    keys = np.zeros(iterations // 10 + 1, dtype=np.int32)
    vals = np.zeros(iterations // 10 + 1)
    nl = I32(0)
    rc = lib().oracle_optimize3(_p(np.ascontiguousarray(row_ptr, np.int64), I64),
                                _p(np.ascontiguousarray(col, np.int32), I32),
                                _p(np.ascontiguousarray(val, np.float64), D), I64(n),
                                _p(Y, D), _p(upd, D), _p(gains, D), C.c_int(METRICS[metric]),
                                D(learning_rate), I32(iterations), D(early_exaggeration),
                                D(initial_momentum), D(final_momentum), D(theta),
                                _p(keys, I32), _p(vals, D), C.byref(nl), C.c_int(threads))
    assert rc == 0
    return dict(zip(keys[:nl.value].tolist(), vals[:nl.value].tolist()))


def repulsion3_queries(Y, theta, Q, threads=1):
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    Q = np.ascontiguousarray(Q, dtype=np.float64)
    rep = np.zeros((Q.shape[0], 3))
    zi = np.zeros(Q.shape[0])
    rc = lib().oracle_repulsion3_queries(_p(Y, D), I64(Y.shape[0]), D(theta), _p(Q, D), I64(Q.shape[0]),
                                         _p(rep, D), _p(zi, D), C.c_int(threads))
    assert rc == 0
    return rep, zi


def attraction3_rows(row_ptr, col, val, Y, rep, Z, r0, r1, metric="sqeuclidean", exaggeration=1.0,
                     want_loss=False):
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    rep = np.ascontiguousarray(rep, dtype=np.float64)
    grad = np.zeros((r1 - r0, 3))
    loss = D(0)
    rc = lib().oracle_attraction3_rows(_p(np.ascontiguousarray(row_ptr, np.int64), I64),
                                       _p(np.ascontiguousarray(col, np.int32), I32),
                                       _p(np.ascontiguousarray(val, np.float64), D), I64(Y.shape[0]),
                                       _p(Y, D), C.c_int(METRICS[metric]), D(exaggeration), _p(rep, D),
                                       D(Z), I64(r0), I64(r1), _p(grad, D),
                                       C.byref(loss) if want_loss else None)
    assert rc == 0
    return grad, (loss.value if want_loss else None)


def project_knn(X, k, metric="sqeuclidean", iterations=3, shifts=None):
    X = np.ascontiguousarray(X, dtype=np.float64)
    n, d = X.shape
    kk = min(k, n - 1)
    idx = np.zeros((n, kk), dtype=np.int32)
    dist = np.zeros((n, kk))
    sh = np.ascontiguousarray(np.asarray(shifts, dtype=np.float64).reshape(max(iterations - 1, 0), d)) \
        if iterations > 1 else None
    rc = lib().oracle_project_knn(_p(X, D), I64(n), I32(d), C.c_int(METRICS[metric]), I32(k), I32(iterations),
                                  _p(sh, D), _p(idx, I32), _p(dist, D))
    assert rc == 0, rc
    return idx, dist
