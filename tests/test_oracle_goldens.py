"""Pin the CPU oracle against every golden vector of the reference's own
test suite (TsneHelpersTestSuite.scala), at the reference's tolerances."""
import numpy as np
import pytest

import oracle_ctypes as O
from golden_data import csr_to_dict, dense_input, goldens, triples_to_csr

G = goldens()


def knn_csr(idx, dist):
    n, k = idx.shape
    return np.arange(0, n * k + 1, k, dtype=np.int64), idx.ravel(), dist.ravel()


def test_knn_bruteforce_golden():
    # TsneHelpersTestSuite.scala:29-42
    X = np.array([v for _, v in G["knnInput"]])
    idx, dist = O.knn(X, 2, "sqeuclidean")
    got = {(i, int(idx[i, t]), float(dist[i, t])) for i in range(9) for t in range(2)}
    want = {tuple(t) for t in G["knnResults"]}
    assert got == want


def test_pairwise_affinities_golden():
    # TsneHelpersTestSuite.scala:76-98: dense_input.csv, k = 10 (> N-1), perplexity 2
    ids, X = dense_input()
    assert list(ids) == list(range(10))
    idx, dist = O.knn(X, 10, "sqeuclidean")
    rp, col, d = knn_csr(idx, dist)
    p, iters = O.affinities(rp, d, 2.0)
    want = {(a, b): c for a, b, c in G["densePairwiseAffinitiesResults"]}
    got = {(i, int(col[e])): p[e] for i in range(10) for e in range(rp[i], rp[i + 1])}
    assert set(got) == set(want)
    for key, v in want.items():
        assert abs(got[key] - v) <= 1e-12, key
    assert iters.max() <= 50


def test_joint_dense_golden():
    # TsneHelpersTestSuite.scala:100-117
    rp, col, val = triples_to_csr(G["densePairwiseAffinitiesResults"], 10)
    orp, oc, ov = O.joint(rp, col, val, 10)
    got = csr_to_dict(orp, oc, ov)
    want = {(a, b): c for a, b, c in G["denseJointProbabilitiesResults"]}
    assert set(got) == set(want)
    for key, v in want.items():
        assert abs(got[key] - v) <= 1e-12
    assert abs(ov.sum() - 1.0) <= 1e-12


def test_joint_sparse_golden():
    # TsneHelpersTestSuite.scala:119-137 (explicit zeros are kept)
    rp, col, val = triples_to_csr(G["sparsePairwiseAffinitiesResults"], 12)
    orp, oc, ov = O.joint(rp, col, val, 12)
    got = csr_to_dict(orp, oc, ov)
    want = {(a, b): c for a, b, c in G["sparseJointProbabilitiesResults"]}
    assert set(got) == set(want)
    for key, v in want.items():
        assert abs(got[key] - v) <= 1e-6
    assert abs(ov.sum() - 1.0) <= 1e-12


def _embedding():
    return np.array([v for _, v in sorted(G["initialEmbedding"])])


def test_gradient_golden_theta0():
    # TsneHelpersTestSuite.scala:168-209
    rp, col, val = triples_to_csr(G["denseJointProbabilitiesResults"], 10)
    r = O.gradient(rp, col, val, _embedding(), theta=0.0)
    want = np.array([v for _, v in sorted(G["denseGradientResults"])])
    assert np.abs(r["grad"] - want).max() <= 1e-12
    # unused goldens, consistent with the code
    assert abs(r["Z"] - G["denseSumQ"]) <= 1e-9


def test_unnormalised_q_golden():
    Y = _embedding()
    for a, b, q in G["denseUnnormLowDimAffinitiesResults"]:
        d = O.lib  # noqa -- metric via numpy, sequential order of 2 terms
        dx, dy = Y[a] - Y[b]
        assert abs(1.0 / (1.0 + (dx * dx + dy * dy)) - q) <= 1e-12


def test_update_golden():
    # TsneHelpersTestSuite.scala:233-271
    Y = _embedding().copy()
    g = np.array([v for _, v in sorted(G["denseGradientResults"])])
    upd = np.zeros_like(Y)
    gains = np.ones_like(Y)
    O.update(g, Y, upd, gains, 0.01, 0.5, 300.0)
    want = np.array([v for _, v in sorted(G["updatedEmbeddingResults"])])
    assert np.abs(Y - want).max() <= 1e-9
    assert np.abs(gains - np.array([v for _, v in sorted(G["updatedGainsResults"])])).max() <= 1e-12
    assert np.abs(upd - np.array([v for _, v in sorted(G["gradientWithMomentumAndGainResults"])])).max() <= 1e-9


def test_iteration_golden():
    # TsneHelpersTestSuite.scala:273-327: one iteration, theta 0, lr 300, momentum 0.5
    rp, col, val = triples_to_csr(G["denseJointProbabilitiesResults"], 10)
    Y = _embedding().copy()
    r = O.gradient(rp, col, val, Y, theta=0.0)
    upd = np.zeros_like(Y)
    gains = np.ones_like(Y)
    O.update(r["grad"], Y, upd, gains, 0.01, 0.5, 300.0)
    O.center(Y)
    want = np.array([v for _, v in sorted(G["updatedAndCentredEmbeddingResults"])])
    assert np.abs(Y - want).max() <= 1e-9


def test_center_golden():
    # TsneHelpersTestSuite.scala:139-166 (exact)
    Y = np.array([v for _, v in sorted(G["centeringInput"])])
    O.center(Y)
    want = np.array([v for _, v in sorted(G["centeringResults"])])
    assert np.array_equal(Y, want)


def test_optimize_matches_manual_schedule():
    """optimize() == iterating gradient/update/centre with the reference
    phase schedule (TsneHelpers.scala:403-427): exaggeration for t <= 101,
    initial momentum for t <= 20, loss every 10 iterations."""
    rp, col, val = triples_to_csr(G["denseJointProbabilitiesResults"], 10)
    Y0 = _embedding() * 1e-3
    T = 110
    Ya, ua, ga = Y0.copy(), np.zeros_like(Y0), np.ones_like(Y0)
    loss = O.optimize(rp, col, val, Ya, ua, ga, learning_rate=100.0, iterations=T,
                      early_exaggeration=4.0, theta=0.25)
    Yb, ub, gb = Y0.copy(), np.zeros_like(Y0), np.ones_like(Y0)
    manual = {}
    for t in range(1, T + 1):
        ex = 4.0 if t <= 101 else 1.0
        mom = 0.5 if t <= 20 else 0.8
        r = O.gradient(rp, col, val, Yb, theta=0.25, exaggeration=ex, want_loss=(t % 10 == 0))
        if t % 10 == 0:
            manual[t] = r["loss"]
        O.update(r["grad"], Yb, ub, gb, 0.01, mom, 100.0)
        O.center(Yb)
    assert np.array_equal(Ya, Yb)
    assert loss == manual
    assert sorted(loss) == list(range(10, T + 1, 10))


def test_bh_reference_criterion_scale_dependence():
    """QuadTree.scala:133-134: max(h)/D < theta with h the HALF width and D
    the SQUARED distance.  Small embeddings are traversed exactly; large
    ones are summarised aggressively."""
    rng = np.random.default_rng(0)
    base = rng.normal(size=(300, 2))
    rp = np.zeros(301, dtype=np.int64)
    none = (np.zeros(0, np.int32), np.zeros(0))
    small = base * 1e-3
    ex = O.gradient(rp, *none, small, theta=0.0)
    bh = O.gradient(rp, *none, small, theta=0.5)
    assert np.abs(bh["rep"] - ex["rep"]).max() <= 1e-9 * np.abs(ex["rep"]).max()
    assert bh["visits"].mean() >= 0.9 * ex["visits"].mean()
    big = base * 50
    ex = O.gradient(rp, *none, big, theta=0.0)
    bh = O.gradient(rp, *none, big, theta=0.5)
    assert bh["visits"].mean() < 0.2 * ex["visits"].mean()


# ----------------------------------------------- 3-D extension (octree restatement)
def _exact3(Y):
    """O(N^2) repulsion sums sum_j (y_i - y_j)/(1+D)^2, sum_j 1/(1+D), j != i."""
    d = Y[:, None, :] - Y[None, :, :]
    D = (d ** 2).sum(-1)
    q = 1.0 / (1.0 + D)
    np.fill_diagonal(q, 0.0)
    return (q[:, :, None] ** 2 * d).sum(1), q.sum(1)


def test_octree_theta0_is_exact():
    """theta = 0 opens every cell: the 3-D restatement equals the exact sums."""
    rng = np.random.default_rng(4)
    Y = rng.normal(size=(400, 3))
    rp = np.zeros(401, dtype=np.int64)
    none = (np.zeros(0, np.int32), np.zeros(0))
    r = O.gradient3(rp, *none, Y, theta=0.0)
    rep, zi = _exact3(Y)
    assert np.abs(r["rep"] - rep).max() <= 1e-12 * np.abs(rep).max()
    assert np.abs(r["zi"] - zi).max() <= 1e-12 * zi.max()


def test_octree_bh_error_shrinks_with_theta():
    rng = np.random.default_rng(5)
    Y = rng.normal(size=(500, 3))
    rp = np.zeros(501, dtype=np.int64)
    none = (np.zeros(0, np.int32), np.zeros(0))
    rep, zi = _exact3(Y)
    err = []
    for theta in (0.5, 0.1, 0.02):
        r = O.gradient3(rp, *none, Y, theta=theta)
        assert abs(r["Z"] - zi.sum()) <= 0.05 * zi.sum()
        err.append(np.abs(r["rep"] - rep).max())
    assert err[0] > err[1] > err[2] and err[2] <= 1e-2 * np.abs(rep).max()


# ----------------------------------------------- projectKnn (Z-order candidates)
def test_project_knn_exact_cases():
    """Two cases where projectKnn provably equals the exact kNN: 1-D
    nonnegative data (Z-order = numeric order, so the k nearest lie within k
    sorted positions on either side) and k >= n-1 (every point a candidate)."""
    rng = np.random.default_rng(2)
    X1 = rng.random((300, 1)) * 10
    pi, pd = O.project_knn(X1, 7, iterations=1)
    ei, ed = O.knn(X1, 7)
    assert np.array_equal(pd, ed) and np.array_equal(pi, ei)
    X2 = rng.random((40, 6))
    pi, pd = O.project_knn(X2, 45, iterations=2, shifts=rng.random((1, 6)))
    ei, ed = O.knn(X2, 45)
    assert np.array_equal(pi, ei) and np.array_equal(pd, ed)


def test_project_knn_recall_improves_with_shifts():
    rng = np.random.default_rng(3)
    X = np.abs(rng.normal(size=(8, 12)))[rng.integers(0, 8, 1500)] * 3 + rng.random((1500, 12))
    ei, _ = O.knn(X, 10)
    rec = []
    for it in (1, 4):
        pi, pd = O.project_knn(X, 10, iterations=it, shifts=rng.random((it - 1, 12)))
        assert (np.diff(pd, axis=1) >= 0).all()
        rec.append(np.mean([len(set(a) & set(b)) / 10 for a, b in zip(pi, ei)]))
    assert rec[1] > rec[0] > 0.2, rec
