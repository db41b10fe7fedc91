"""The library's own multi-rank (world > 1) path, executed on ONE GPU.

optimize.hip with world > 1: rank r owns a range of internal labels (rows of
P); every rank builds the same tree from the full embedding, runs BH for its
own points only (its query list in Morton order) and the attraction + update
for its rows; per iteration only Z (all-reduce of one double) and the updated
embedding slices (ragged all-gather) cross ranks, plus the loss every 10th
iteration and, at a relabel, the bucket costs and the momentum/gains slices.

Two ways to run it without 8 GPUs:
  * tsne_ctx_create_multi with a repeated device id: loopback ranks, one host
    thread each, inside one process (the single-caller multi-device entry a
    Flink operator at parallelism 1 uses; RCCL when the devices differ);
  * tsne_ctx_init_comm_callbacks: the collectives carried by the caller --
    here torch.distributed over gloo, two processes sharing the GPU.

Against the world = 1 trajectory.  Bit-equality is not expected: a query's
BH sums are accumulated in an order that depends on which queries share its
wave (batch pops of the wave-shared stack), and a rank's waves are formed from
its own queries; Z is summed per rank.  Both are rounding-level (~1e-16
relative) and the reference dynamics are chaotic, so the tolerance is 1e-9
relative over 60 iterations (two Morton relabel checks, one cost-balanced
re-cut) -- far below the 1e-4 gradient bar.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_ctypes as O
import tsne_amd as T
from tsne_amd.api import default_params

pytestmark = pytest.mark.gpu

TOL = 1e-9


def problem(n=1500, k=30, seed=5, c=2, scale=1e-3):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(6, 10))[rng.integers(0, 6, n)] * 6 + rng.normal(size=(n, 10))
    idx, d = O.knn(X, k)
    rp = np.arange(0, n * k + 1, k, dtype=np.int64)
    p, _ = O.affinities(rp, d.ravel(), k / 3)
    P = O.joint(rp, idx.ravel(), p, n)
    Y0 = rng.normal(size=(n, c)) * scale
    return P, Y0


def run_single(P, Y0, params):
    with T.Context(0) as ctx:
        Y, u, g = Y0.copy(), np.zeros_like(Y0), np.ones_like(Y0)
        loss = ctx.optimize(*P, Y, u, g, params)
    return Y, u, g, loss


def close(a, b):
    return np.abs(a - b).max() <= TOL * max(1.0, np.abs(b).max())


@pytest.mark.parametrize("world", [2, 3])
def test_multi_knn_split_matches_single(world):
    X = np.random.default_rng(world).normal(size=(1700, 24))
    with T.Context(0) as one:
        i1, d1 = one.kNearestNeighbors(X, 20)
    m = T.Context.multi([0] * world)
    try:
        assert m.rank_world() == (0, world)
        im, dm = m.kNearestNeighbors(X, 20)
    finally:
        m.close()
    assert np.array_equal(i1, im) and np.array_equal(d1, dm)


@pytest.mark.parametrize("world", [2, 3])
def test_multi_optimize_loopback_matches_single(world):
    P, Y0 = problem()
    prm = default_params(iterations=60, theta=0.5, learning_rate=200.0)
    Ys, us, gs, ls = run_single(P, Y0, prm)
    m = T.Context.multi([0] * world)
    try:
        Y, u, g = Y0.copy(), np.zeros_like(Y0), np.ones_like(Y0)
        lm = m.optimize(*P, Y, u, g, prm)
    finally:
        m.close()
    assert sorted(lm) == sorted(ls) == list(range(10, 61, 10))
    for t in ls:
        assert abs(lm[t] - ls[t]) <= TOL * abs(ls[t]), (t, lm[t], ls[t])
    assert close(Y, Ys) and close(u, us) and close(g, gs)


def test_multi_optimize_loopback_serial_timing():
    """Option loop_serial (comm.cpp LoopGroup): the ranks take turns on the
    device and log each stretch of work between collectives, with the tree /
    BH phase marks -- the same results as world 1, and a summary
    (tsne_ctx_loop_profile) whose per-collective counts follow the schedule
    (scripts/loop_projection.py)."""
    P, Y0 = problem()
    prm = default_params(iterations=40, theta=0.5, learning_rate=200.0)
    Ys, _, _, ls = run_single(P, Y0, prm)
    m = T.Context.multi([0, 0])
    try:
        m.set_option("loop_serial", 1)
        Y, u, g = Y0.copy(), np.zeros_like(Y0), np.ones_like(Y0)
        lm = m.optimize(*P, Y, u, g, prm)
        rep = m.loop_profile()
        again = m.loop_profile()
    finally:
        m.close()
    for t in ls:
        assert abs(lm[t] - ls[t]) <= TOL * abs(ls[t]), t
    assert close(Y, Ys)
    assert again["segments"] == 0   # a read clears the log
    assert rep["world"] == 2 and len(rep["rank_total_ms"]) == 2 and rep["span_ms"] > 0
    lab = rep["by_collective"]
    # one Z all-reduce per iteration + the loss every 10th; one Y all-gather per iteration
    # (+ the gathers of a relabel); a tree and a BH mark per iteration
    assert lab["allreduce_f64[1]"]["count"] >= 40 + 4
    assert lab["allgatherv"]["count"] >= 40
    marks = sum(v["count"] for k, v in lab.items() if k.startswith("tree"))
    assert marks == 40 and sum(v["count"] for k, v in lab.items() if k.startswith("bh")) == 40
    assert all(v["max_ms"] >= v["mean_ms"] >= 0 for v in lab.values())


def test_multi_optimize3_loopback_matches_single():
    P, Y0 = problem(n=900, c=3, seed=8)
    prm = default_params(n_components=3, iterations=40, theta=0.5, learning_rate=200.0)
    Ys, us, gs, ls = run_single(P, Y0, prm)
    m = T.Context.multi([0, 0])
    try:
        Y, u, g = Y0.copy(), np.zeros_like(Y0), np.ones_like(Y0)
        lm = m.optimize(*P, Y, u, g, prm)
    finally:
        m.close()
    assert sorted(lm) == sorted(ls)
    for t in ls:
        assert abs(lm[t] - ls[t]) <= TOL * abs(ls[t]), t
    assert close(Y, Ys) and close(u, us) and close(g, gs)


def test_multi_rejects_mixed_devices():
    with pytest.raises(T.TsneError) as e:
        T.Context.multi([0, 0, 1])
    assert e.value.status == -1


def test_multi_handle_refuses_device_optimizer():
    """tsne_dev_opt_* hold one rank's state: on a handle of two loopback ranks
    they fail with TSNE_ERR_UNSUPPORTED instead of rank 0 waiting forever in
    a collective for a rank that never calls in (tsne_optimize is the
    multi-rank form)."""
    n = 256
    rng = np.random.default_rng(3)
    rp = np.arange(0, n * 4 + 1, 4, dtype=np.int64)
    dev = torch.device("cuda", 0)
    Pd = (torch.from_numpy(rp).to(dev), torch.from_numpy(rng.integers(0, n, n * 4).astype(np.int32)).to(dev),
          torch.full((n * 4,), 1.0 / (n * 4), dtype=torch.float64, device=dev))
    Y = torch.from_numpy(rng.normal(size=(n, 2)) * 1e-4).to(dev)
    m = T.Context.multi([0, 0])
    try:
        with pytest.raises(T.TsneError) as e:
            m.dev_opt_setup(default_params(iterations=10), *Pd, n, Y, torch.zeros_like(Y), torch.ones_like(Y))
        assert e.value.status == -4
        with pytest.raises(T.TsneError) as e:
            m.dev_opt_step(1)
        assert e.value.status == -4
    finally:
        m.close()


# ------------------------------------------ caller-supplied collectives (gloo)
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, out_path, T_):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root / "tsne-flink_amd"))
    sys.path.insert(0, str(root / "tests"))
    import tsne_amd as TA
    from tsne_amd.api import default_params as dp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    P, Y0 = problem()

    def allreduce_sum(a):
        t = torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a)
        dist.all_reduce(t)

    def allgatherv(buf, off):
        for r in range(world):
            seg = torch.from_numpy(buf[off[r]:off[r + 1]])
            if seg.numel():
                dist.broadcast(seg, src=r)

    with TA.Context(0) as ctx:
        ctx.init_comm_callbacks(rank, world, allreduce_sum, allgatherv)
        assert ctx.rank_world() == (rank, world)
        Y, u, g = Y0.copy(), np.zeros_like(Y0), np.ones_like(Y0)
        loss = ctx.optimize(*P, Y, u, g, dp(iterations=T_, theta=0.5, learning_rate=200.0))
    if rank == 0:
        np.savez(out_path, Y=Y, u=u, g=g, keys=np.array(sorted(loss)),
                 vals=np.array([loss[k] for k in sorted(loss)]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_callbacks_world2_matches_single(tmp_path):
    """Two processes on the GPU, the library's world = 2 optimizer with its
    collectives carried by torch.distributed (gloo) through
    tsne_ctx_init_comm_callbacks -- the replay of test_sharded_gloo.py with the
    library, not the oracle, doing the compute."""
    T_ = 60
    out = tmp_path / "gloo.npz"
    mp.start_processes(_gloo_worker, args=(2, _free_port(), str(out), T_), nprocs=2, start_method="spawn",
                       join=True)
    res = np.load(out)
    P, Y0 = problem()
    Ys, us, gs, ls = run_single(P, Y0, default_params(iterations=T_, theta=0.5, learning_rate=200.0))
    assert list(res["keys"]) == sorted(ls)
    for k, v in zip(res["keys"], res["vals"]):
        assert abs(v - ls[int(k)]) <= TOL * abs(ls[int(k)])
    assert close(res["Y"], Ys) and close(res["u"], us) and close(res["g"], gs)


# ------------------------------------------------ RCCL transport at world 1
def _world1_run(P, Y0, prm, transport):
    """The sharded optimizer (query lists, collectives, centring from the
    gathered embedding) at world 1 through a forced communicator
    (Options::comm_world1): RCCL (a one-rank ncclCommInitRankConfig) or the
    caller's callbacks (identity collectives)."""
    ctx = T.Context(0)
    try:
        ctx.set_option("comm_world1", 1)
        if transport == "rccl":
            ctx.init_comm(0, 1, None)
        else:
            ctx.init_comm_callbacks(0, 1, lambda a: None, lambda buf, off: None)
        assert ctx.rank_world() == (0, 1)
        kind = ctx.counter("comm.kind")
        Y, u, g = Y0.copy(), np.zeros_like(Y0), np.ones_like(Y0)
        loss = ctx.optimize(*P, Y, u, g, prm)
        calls = ctx.counter("comm.calls")
    finally:
        ctx.close()
    return Y, u, g, loss, kind, calls


@pytest.mark.parametrize("c", [2, 3])
def test_rccl_world1_sharded_path_matches_callbacks(c):
    """RCCL's ncclAllReduce and the ncclBroadcast group of the ragged all-gather
    execute in the optimizer's sharded path (one rank): bit-identical to the
    same path through identity callbacks, and within the multi-rank tolerance
    of the unsharded world-1 run (summation order of the query-list Z)."""
    P, Y0 = problem(n=1200 if c == 2 else 800, c=c, seed=11)
    prm = default_params(n_components=c, iterations=40, theta=0.5, learning_rate=200.0)
    Yr, ur, gr, lr, kr, nr = _world1_run(P, Y0, prm, "rccl")
    Yc, uc, gc, lc, kc, nc = _world1_run(P, Y0, prm, "callbacks")
    assert (kr, kc) == (1, 3)
    assert nr == nc and nr >= 40 + 40   # a Z all-reduce and a Y all-gather per iteration, at least
    assert np.array_equal(Yr, Yc) and np.array_equal(ur, uc) and np.array_equal(gr, gc)
    assert lr == lc
    Ys, us, gs, ls = run_single(P, Y0, prm)
    for t in ls:
        assert abs(lr[t] - ls[t]) <= TOL * abs(ls[t]), t
    assert close(Yr, Ys) and close(ur, us) and close(gr, gs)


# ------------------------------------------------------ tree partition (bh_split)
def _run_opts(P, Y0, prm, world, opts):
    h = T.Context(0) if world == 1 else T.Context.multi([0] * world)
    try:
        for k_, v_ in opts.items():
            h.set_option(k_, v_)
        Y, u, g = Y0.copy(), np.zeros_like(Y0), np.ones_like(Y0)
        loss = h.optimize(*P, Y, u, g, prm)
    finally:
        h.close()
    return Y, u, g, loss


@pytest.mark.parametrize("world,opts", [(3, {"bh_split": 1, "root_tile": 0}), (4, {"bh_split": 1}),
                                        (5, {"bh_split": 1, "root_tile": 0, "relabel": 0}), (2, {"bh_split": 0})])
def test_tree_partition_matches_single(world, opts):
    """Options::bh_split = 1: every rank walks every query over the cells
    holding its own sorted points; shared cells straddle the cuts, their terms
    taken by the owner of their first point, and a shared cell that tiles for
    a lane is summed exactly as the sum of its parts over the ranks
    (REF_FORCED).  root_tile = 0 runs the full tree from t = 1, where the
    tiny embedding makes the root a near-exact tile for every query: the
    forced path from the root down.  Exact duplicate groups included (the
    reference's multiplicities).  Within the multi-rank tolerance of world 1."""
    P, Y0 = problem(n=2000, seed=12)
    Y0 = Y0.copy()
    Y0[100:110] = Y0[7]          # a duplicate group of 11
    Y0[1500:1503] = Y0[900]      # and one of 4
    prm = default_params(iterations=60, theta=0.5, learning_rate=200.0)
    base = {k_: v_ for k_, v_ in opts.items() if k_ != "bh_split"}
    Ys, us, gs, ls = _run_opts(P, Y0, prm, 1, base)
    Y, u, g, lm = _run_opts(P, Y0, prm, world, opts)
    assert sorted(lm) == sorted(ls)
    for t in ls:
        assert abs(lm[t] - ls[t]) <= TOL * abs(ls[t]), (t, lm[t], ls[t])
    assert close(Y, Ys) and close(u, us) and close(g, gs)
