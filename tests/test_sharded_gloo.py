"""The N>1 decomposition on CPU: world_size 2/3 over gloo.

libtsne_hip's multi-GPU iteration (optimize.hip, world > 1): rank r owns a
range of point labels = rows of P (cost-balanced cuts, re-cut from measured
per-bucket costs when the labels are renumbered: tsne_balance_cuts, identical
on every rank after an all-reduce of the costs); every rank builds the same
tree from the full Y and computes BH repulsion for ITS OWN points only; Z is
the all-reduce of the ranks' partial sums (one double); rank r runs attraction
+ update for its rows; the updated Y slices are all-gathered (ragged: one
broadcast per rank); every rank centres; the loss every 10th iteration is one
more all-reduce.  No per-point force crosses ranks.  This test replays exactly
that decomposition with the oracle as the compute and torch.distributed
(gloo) as the exchange, and checks it reproduces the single-process reference
iteration.  (The library's own world > 1 step runs in tests/test_gpu_multi.py,
with loopback ranks and with gloo-carried collectives.)
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_ctypes as O


def _problem(n=300, k=20, seed=3):
    rng = np.random.default_rng(seed)
    X = rng.normal(size=(4, 8))[rng.integers(0, 4, n)] * 4 + rng.normal(size=(n, 8))
    idx, d = O.knn(X, k)
    rp = np.arange(0, n * k + 1, k, dtype=np.int64)
    p, _ = O.affinities(rp, d.ravel(), k / 3)
    P = O.joint(rp, idx.ravel(), p, n)
    Y = rng.normal(size=(n, 2)) * 1e-2
    return P, Y


def _worker(rank, world, port, T, out_path):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root / "tsne-flink_amd"))
    sys.path.insert(0, str(root / "tests"))
    import oracle_ctypes as Ow
    import tsne_amd as TA
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    (rp, col, val), Y = _problem()
    n = Y.shape[0]
    upd, gains = np.zeros_like(Y), np.ones_like(Y)
    losses = {}
    BUCKET = 16
    cut_log = []
    nb = -(-n // BUCKET)
    own = np.array([min(n, -(-n // world) * r) for r in range(world + 1)], dtype=np.int64)
    for t in range(1, T + 1):
        ex = 4.0 if t <= 101 else 1.0
        mom = 0.5 if t <= 20 else 0.8
        r0, r1 = int(own[rank]), int(own[rank + 1])
        # BH for this rank's own points only
        rep = np.zeros((n, 2))
        cost = np.zeros(nb, dtype=np.uint64)
        zpart = np.zeros(1)
        if r1 > r0:
            rep_s, z_s = Ow.repulsion_queries(Y, 0.5, Y[r0:r1])
            rep[r0:r1] = rep_s
            zpart[0] = z_s.sum()
            # any per-query cost measured on the slice will do; the library uses its wave times
            vis = (1 + 100.0 * np.abs(rep_s).sum(1) / max(1e-300, np.abs(rep_s).sum(1).max())).astype(np.uint64)
            np.add.at(cost, np.arange(r0, r1) // BUCKET, vis)
        zt = torch.from_numpy(zpart)
        dist.all_reduce(zt)                                    # the only per-iteration all-reduce
        Z = float(zt.item())
        g, lpart = Ow.attraction_rows(rp, col, val, Y, rep, Z, r0, r1, exaggeration=ex,
                                      want_loss=(t % 10 == 0))
        Yr, ur, gr = Y[r0:r1].copy(), upd[r0:r1].copy(), gains[r0:r1].copy()
        Ow.update(np.ascontiguousarray(g), Yr, ur, gr, 0.01, mom, 200.0)
        upd[r0:r1], gains[r0:r1] = ur, gr
        Ynew = Y.copy()
        Ynew[r0:r1] = Yr
        for r in range(world):                                 # ragged all-gather: one broadcast per rank
            seg = torch.from_numpy(np.ascontiguousarray(Ynew[own[r]:own[r + 1]]))
            if seg.numel():
                dist.broadcast(seg, src=r)
                Ynew[own[r]:own[r + 1]] = seg.numpy()
        Y = Ynew
        Ow.center(Y)
        if t % 10 == 0:
            lt = torch.tensor([lpart], dtype=torch.float64)
            dist.all_reduce(lt)
            losses[t] = float(lt.item())
            # re-cut the ownership by the measured costs (the library does this at
            # its relabels); the rows' momentum / gains follow their new owner
            ct = torch.from_numpy(cost.astype(np.int64))
            dist.all_reduce(ct)
            for r in range(world):
                for a in (upd, gains):
                    seg = torch.from_numpy(np.ascontiguousarray(a[own[r]:own[r + 1]]))
                    if seg.numel():
                        dist.broadcast(seg, src=r)
                        a[own[r]:own[r + 1]] = seg.numpy()
            own = TA.balance_cuts(ct.numpy().astype(np.uint64), n, world, bucket=BUCKET)
            if rank == 0:
                cut_log.append(own.tolist())
    if rank == 0:
        np.savez(out_path, Y=Y, keys=np.array(sorted(losses)), vals=np.array([losses[k] for k in sorted(losses)]),
                 cuts=np.array(cut_log))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_iteration_matches_single_process(tmp_path, world):
    T = 30
    out = tmp_path / "sharded.npz"
    mp.start_processes(_worker, args=(world, _free_port(), T, str(out)), nprocs=world,
                       start_method="spawn", join=True)
    res = np.load(out)
    (rp, col, val), Y = _problem()
    upd, gains = np.zeros_like(Y), np.ones_like(Y)
    ref = O.optimize(rp, col, val, Y, upd, gains, learning_rate=200.0, iterations=T, theta=0.5)
    assert list(res["keys"]) == sorted(ref)
    for k, v in zip(res["keys"], res["vals"]):
        assert abs(v - ref[int(k)]) <= 1e-9 * abs(ref[int(k)])
    assert np.abs(res["Y"] - Y).max() <= 1e-9 * np.abs(Y).max()
    cuts = res["cuts"]
    assert (np.diff(cuts, axis=1) >= 0).all() and (cuts[:, 0] == 0).all() and (cuts[:, -1] == Y.shape[0]).all()
    assert len({tuple(c) for c in cuts}) > 1        # the cuts follow the measured costs


def test_balance_cuts_rule():
    """tsne_balance_cuts (host mirror of the device rule in bhtree.hip)."""
    import tsne_amd as TA
    assert TA.balance_cuts([0, 0, 0, 0], 1000, 4).tolist() == [0, 250, 500, 750, 1000]
    assert TA.balance_cuts([1, 1, 1, 1], 1000, 2).tolist() == [0, 512, 1000]
    assert TA.balance_cuts([100, 1, 1, 1], 1000, 2).tolist() == [0, 256, 1000]
    assert TA.balance_cuts([1], 10, 8).tolist() == [0, 0, 0, 0, 0, 0, 0, 0, 10]
    rng = np.random.default_rng(0)
    c = rng.integers(0, 1000, 500)
    b = TA.balance_cuts(c, 500 * 256 - 7, 8)
    pre = np.concatenate([[0], np.cumsum(c)])
    for r in range(1, 8):
        k = b[r] // 256
        assert pre[k] >= c.sum() * r // 8 > pre[k - 1]


def _worker3(rank, world, port, T, out_path):
    """The 3-D (octree) decomposition of optimize.hip opt_step3: equal label
    ranges (= rows of P, no relabelling), BH for the rank's own points, Z
    all-reduced, ragged all-gather of the Y slices, local centring."""
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root / "tsne-flink_amd"))
    sys.path.insert(0, str(root / "tests"))
    import oracle_ctypes as Ow
    import tsne_amd as TA
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    (rp, col, val), _ = _problem()
    Y = np.random.default_rng(8).normal(size=(rp.shape[0] - 1, 3)) * 1e-2
    n = Y.shape[0]
    r0, r1 = TA.shard_rows(n, world, rank)
    upd, gains = np.zeros_like(Y), np.ones_like(Y)
    losses = {}
    for t in range(1, T + 1):
        ex = 4.0 if t <= 101 else 1.0
        mom = 0.5 if t <= 20 else 0.8
        rep = np.zeros((n, 3))
        zpart = np.zeros(1)
        if r1 > r0:
            rep_s, z_s = Ow.repulsion3_queries(Y, 0.5, Y[r0:r1])
            rep[r0:r1] = rep_s
            zpart[0] = z_s.sum()
        zt = torch.from_numpy(zpart)
        dist.all_reduce(zt)
        Z = float(zt.item())
        g, lpart = Ow.attraction3_rows(rp, col, val, Y, rep, Z, r0, r1, exaggeration=ex, want_loss=(t % 10 == 0))
        Yr, ur, gr = Y[r0:r1].copy(), upd[r0:r1].copy(), gains[r0:r1].copy()
        Ow.update(np.ascontiguousarray(g), Yr, ur, gr, 0.01, mom, 200.0)
        upd[r0:r1], gains[r0:r1] = ur, gr
        Ynew = Y.copy()
        Ynew[r0:r1] = Yr
        for r in range(world):
            a0, a1 = TA.shard_rows(n, world, r)
            seg = torch.from_numpy(np.ascontiguousarray(Ynew[a0:a1]))
            if seg.numel():
                dist.broadcast(seg, src=r)
                Ynew[a0:a1] = seg.numpy()
        Y = Ynew
        Ow.center(Y)
        if t % 10 == 0:
            lt = torch.tensor([lpart], dtype=torch.float64)
            dist.all_reduce(lt)
            losses[t] = float(lt.item())
    if rank == 0:
        np.savez(out_path, Y=Y, keys=np.array(sorted(losses)), vals=np.array([losses[k] for k in sorted(losses)]))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_octree_iteration_matches_single_process(tmp_path):
    T, world = 20, 2
    out = tmp_path / "sharded3.npz"
    mp.start_processes(_worker3, args=(world, _free_port(), T, str(out)), nprocs=world,
                       start_method="spawn", join=True)
    res = np.load(out)
    (rp, col, val), _ = _problem()
    Y = np.random.default_rng(8).normal(size=(rp.shape[0] - 1, 3)) * 1e-2
    upd, gains = np.zeros_like(Y), np.ones_like(Y)
    ref = O.optimize3(rp, col, val, Y, upd, gains, learning_rate=200.0, iterations=T, theta=0.5)
    assert list(res["keys"]) == sorted(ref)
    for k, v in zip(res["keys"], res["vals"]):
        assert abs(v - ref[int(k)]) <= 1e-9 * abs(ref[int(k)])
    assert np.abs(res["Y"] - Y).max() <= 1e-9 * np.abs(Y).max()
