"""bench.py's CPU-side pieces (no GPU): the CPU baseline leg (the oracle's
tree built once, queries timed apart) and the reference tree handle it uses."""
import argparse

import numpy as np
import torch

import oracle_ctypes as O


def test_tree_handle_matches_repulsion_queries():
    rng = np.random.default_rng(3)
    for scale in (1e-4, 1.0, 20.0):
        Y = rng.normal(size=(3000, 2)) * scale
        Y[7] = Y[11]                                    # a duplicate pair
        Q = Y[rng.choice(3000, 200, replace=False)]
        tree = O.Tree(Y)
        r1, z1, v = tree.query(0.5, Q, threads=4)
        r2, z2 = O.repulsion_queries(Y, 0.5, Q, threads=1)
        tree.close()
        assert np.array_equal(r1, r2) and np.array_equal(z1, z2)
        assert v >= len(Q)


def test_cpu_baseline_block():
    import bench
    rng = np.random.default_rng(0)
    n, k = 2000, 30
    X = rng.normal(size=(n, 8))
    idx, dist = O.knn(X, k)
    rp = np.arange(0, n * k + 1, k, dtype=np.int64)
    p, _ = O.affinities(rp, dist.ravel(), 10.0)
    jr, jc, jv = O.joint(rp, idx.ravel(), p, n)
    snaps = {t: rng.normal(size=(n, 2)) * s for t, s in ((1, 1e-4), (100, 1.0), (1000, 30.0))}
    a = argparse.Namespace(theta=0.5, iterations=1000, cpu_budget=0.05, k=k, cpu_knn_sample=8)
    out, detail = bench.cpu_baseline(snaps, a, n, X, (torch.from_numpy(jr), torch.from_numpy(jc),
                                                       torch.from_numpy(jv)))
    assert out["kind"] == "port" and out["value"] > 0 and out["knn_pts_per_s"] > 0
    assert set(out["per_iteration_s_at"]) == {"1", "100", "1000"}
    for t in ("1", "100", "1000"):
        assert detail[t]["queries"] >= 2 * 16 and detail[t]["build_s"] > 0
    # the near-exact early snapshot does more reference work per query than the
    # late one (counted, not timed: at n = 2000 the timings are within noise)
    assert all(out["per_iteration_s_at"][t] > 0 for t in ("1", "100", "1000"))
    assert detail["1"]["visits_per_query"] > detail["1000"]["visits_per_query"]
