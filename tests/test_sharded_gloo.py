"""The N>1 decomposition on CPU: world_size 2 over gloo.

libtsne_hip's multi-GPU iteration (optimize.hip) is: every rank builds the
same tree from the full Y; rank r computes BH repulsion for its contiguous
slice of the Morton-sorted points; the (F, z) slices are all-gathered; Z is
summed locally; rank r runs attraction + update for its rows of P
(tsne_shard_rows); the updated Y slices are all-gathered; every rank centres.
This test replays exactly that decomposition with the oracle as the compute
and torch.distributed (gloo) as the exchange, and checks it reproduces the
single-process reference iteration.  The slicing comes from the library's
own host logic (tsne_shard_rows), which needs no GPU.
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


def _sorted_order(Y):
    # any fixed permutation shared by all ranks stands in for the Morton order
    return np.lexsort((Y[:, 1], Y[:, 0]))


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
    r0, r1 = TA.shard_rows(n, world, rank)
    chunk = -(-n // world)
    upd, gains = np.zeros_like(Y), np.ones_like(Y)
    losses = {}
    for t in range(1, T + 1):
        ex = 4.0 if t <= 101 else 1.0
        mom = 0.5 if t <= 20 else 0.8
        # BH for this rank's slice of the sorted order
        order = _sorted_order(Y)
        sl = order[r0:r1]
        rep_s, z_s = Ow.repulsion_queries(Y, 0.5, Y[sl])
        buf = np.zeros((chunk, 3))
        buf[: r1 - r0, :2] = rep_s
        buf[: r1 - r0, 2] = z_s
        gathered = [torch.zeros(chunk, 3, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(gathered, torch.from_numpy(buf))
        full = torch.cat(gathered).numpy()[:n]
        rep = np.zeros((n, 2))
        z = np.zeros(n)
        rep[order] = full[:, :2]
        z[order] = full[:, 2]
        Z = z.sum()
        g, lpart = Ow.attraction_rows(rp, col, val, Y, rep, Z, r0, r1, exaggeration=ex,
                                      want_loss=(t % 10 == 0))
        Yr, ur, gr = Y[r0:r1].copy(), upd[r0:r1].copy(), gains[r0:r1].copy()
        Ow.update(np.ascontiguousarray(g), Yr, ur, gr, 0.01, mom, 200.0)
        upd[r0:r1], gains[r0:r1] = ur, gr
        ybuf = np.zeros((chunk, 2))
        ybuf[: r1 - r0] = Yr
        gy = [torch.zeros(chunk, 2, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(gy, torch.from_numpy(ybuf))
        Y = np.ascontiguousarray(torch.cat(gy).numpy()[:n])
        Ow.center(Y)
        if t % 10 == 0:
            lt = torch.tensor([lpart], dtype=torch.float64)
            dist.all_reduce(lt)
            losses[t] = float(lt.item())
    if rank == 0:
        np.savez(out_path, Y=Y, keys=np.array(sorted(losses)), vals=np.array([losses[k] for k in sorted(losses)]))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2])
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
