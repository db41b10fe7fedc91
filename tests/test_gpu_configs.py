"""Every BASELINE.json config at its full size, against the oracle.

Full-size runs are checked where the oracle finishes in seconds -- sampled
query rows / gradient rows of the real pipeline, plus size-independent
identities -- and end to end where the whole problem is small (C1):

  C1  2,000 x 50, perplexity 30, 300 iterations, theta 0.25, lr 1000: the
      native CLI end to end (COO file in, CSV + loss file out) against the
      oracle pipeline from the same seeded Y0 (loss keys, early KL at 1 %, the
      final KL inside the oracle's own perturbation ensemble: DESIGN.md 4);
  C2  70,000 x 784 MNIST-shaped, theta 0.5, T = 1000;
  C3  1,000,000 x 128 GMM, theta 0.5, T = 1000 (the bench workload);
  C4  500,000 x 300 sparse, cosine, nComponents 3 (octree extension);
  C5  precomputed distance matrix (--inputDistanceMatrix): the CLI end to end
      at 2,000 points (with and without the diagonal) and the library at
      5,000 points against the oracle (the 50,000-point run is a bench mode:
      bench.py --config c5).  Dense rows underflow to p = 0, so the
      reference's KL is NaN (0 ln 0, TsneHelpers.scala:300) -- reproduced
      exactly (same loss keys, NaN at the same iterations); the KL over the
      support P > 0 is compared instead;
  C2-C4 each: kNN rows bit-exact (256 contiguous query rows vs oracle_knn),
      affinity rows at 1e-12, joint rows (pattern exact, values 1e-13
      relative) against a restatement of jointDistribution on the sampled
      rows, and at snapshots of the real optimizer trajectory the per-point
      repulsion (z at the library's near-exact bound "near_tol_early" = 1e-6
      relative; the gradient of a row block at 1e-4 x max|grad| and, per row
      with |g_i| >= 1e-3 max|g|, at 1e-4 x |g_i|: north_star's "per-iteration
      gradients within 1e-4 relative"; the measured per-row figures go to
      gpurun_out/grad_row_rel.json), Z == sum of the per-point z, and the KL
      loss over all rows at 1e-9 (the oracle's attraction + loss with the same
      Z).
"""
import json
import math
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest
import torch

import configs as CF
import oracle_ctypes as O
import tsne_amd as T
from tsne_amd.api import default_params

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
CLI = ROOT / "tsne-flink_amd" / "tsne_hip"
THREADS = 16
ROW_REL = {}   # config/snapshot -> measured per-row relative gradient error (written to gpurun_out/)


def near_tol(c, late=False):
    """The library's near-exact bound, read from the context: single gradients
    (tsne_gradient / tsne_repulsion) and the optimizer's exaggerated phase run
    at "near_tol_early", the optimizer after it at "near_tol_late"."""
    return c.get_option("near_tol_late" if late else "near_tol_early")


def row_relative(g, g_ref, key):
    """max over rows with |g_i| >= 1e-3 max|g| of |g_i - g_ref_i| / |g_ref_i|
    (2-norms per row); recorded under `key` and returned."""
    nrm = np.linalg.norm(g_ref, axis=1)
    sel = nrm >= 1e-3 * nrm.max()
    rel = float((np.linalg.norm(g - g_ref, axis=1)[sel] / nrm[sel]).max())
    ROW_REL[key] = {"max_row_rel": rel, "rows": int(sel.sum()), "of": int(len(nrm))}
    out = ROOT / "gpurun_out"
    out.mkdir(exist_ok=True)
    (out / "grad_row_rel.json").write_text(json.dumps(ROW_REL, indent=1, sort_keys=True))
    return rel


@pytest.fixture(scope="module")
def ctx():
    c = T.Context(0)
    yield c
    c.close()


def exaggeration(t, T_=1000):
    return 4.0 if t <= min(T_, 20) + min(max(T_ - 20, 0), 81) else 1.0


# ------------------------------------------------------------------ helpers
def check_knn_rows(X_host, idx, dist, k, metric, q0, nq=256):
    oi, od = O.knn(X_host, k, metric, q0=q0, q1=q0 + nq, threads=THREADS)
    assert np.array_equal(idx[q0:q0 + nq], oi), "kNN ids"
    assert np.array_equal(np.isnan(dist[q0:q0 + nq]), np.isnan(od))
    assert np.array_equal(np.nan_to_num(dist[q0:q0 + nq]), np.nan_to_num(od)), "kNN distances"


def check_affinity_rows(dist, p, perplexity, rows):
    k = dist.shape[1]
    rp = np.arange(0, len(rows) * k + 1, k, dtype=np.int64)
    po, _ = O.affinities(rp, dist[rows].ravel(), perplexity)
    assert np.abs(p[rows].ravel() - po).max() <= 1e-12


def check_joint_rows(idx, p, orp, oc, ov, rows):
    """jointDistribution (TsneHelpers.scala:182-196) restated for single rows:
    J_ij = p_j|i + p_i|j over the union pattern, P = J / sum(J), sum(J) = 2 sum(p)."""
    tot = 2.0 * p.sum()
    flat_i = idx.ravel()
    for i in rows:
        want = {}
        for j, v in zip(idx[i].tolist(), p[i].tolist()):
            want[j] = want.get(j, 0.0) + v
        for e in np.nonzero(flat_i == i)[0].tolist():
            j = e // idx.shape[1]
            want[j] = want.get(j, 0.0) + p.ravel()[e]
        a, b = orp[i], orp[i + 1]
        got = dict(zip(oc[a:b].tolist(), ov[a:b].tolist()))
        assert set(got) == set(want), i
        assert list(oc[a:b]) == sorted(want), i          # rows sorted by column
        for j, v in want.items():
            assert abs(got[j] - v / tot) <= 1e-13 * (v / tot), (i, j)


def check_gradient_snapshot(ctx, P, Y, theta, ex, metric, r0, nr, c=2, loss=True, key="snapshot"):
    rp, col, val = P
    n = Y.shape[0]
    F, z = ctx.repulsion(Y, theta)
    g, Z, L = ctx.gradient(rp, col, val, Y, theta, metric, exaggeration=ex, want_loss=loss)
    assert abs(Z - z.sum()) <= 1e-12 * Z, (Z, z.sum())
    Q = np.ascontiguousarray(Y[r0:r0 + nr])
    if c == 2:
        rep_o, z_o = O.repulsion_queries(Y, theta, Q, threads=THREADS)
    else:
        rep_o, z_o = O.repulsion3_queries(Y, theta, Q, threads=THREADS)
    assert np.abs(z[r0:r0 + nr] - z_o).max() <= near_tol(ctx) * z_o.max(), "per-point z"
    rep = np.zeros((n, c))
    rep[r0:r0 + nr] = rep_o
    attr = O.attraction_rows if c == 2 else O.attraction3_rows
    g_o, _ = attr(rp, col, val, Y, rep, Z, r0, r0 + nr, metric=metric, exaggeration=ex)
    assert np.abs(g[r0:r0 + nr] - g_o).max() <= 1e-4 * np.abs(g_o).max(), "gradient rows"
    rel = row_relative(g[r0:r0 + nr], g_o, key)
    assert rel <= 1e-4, (key, "per-row relative gradient", rel)
    if loss:
        _, l_o = attr(rp, col, val, Y, np.zeros((n, c)), Z, 0, n, metric=metric, exaggeration=ex, want_loss=True)
        assert abs(L - l_o) <= 1e-9 * abs(l_o), (L, l_o)


def pipeline(ctx, Xd, k, metric, perplexity):
    """kNN -> affinities -> joint on the device (the bench's path); host copies."""
    n = Xd.shape[0]
    kk = min(k, n - 1)
    dev = Xd.device
    idx = torch.empty((n, kk), dtype=torch.int32, device=dev)
    dist = torch.empty((n, kk), dtype=torch.float64, device=dev)
    ctx.dev_knn(Xd, k, metric, 0, n, idx, dist)
    rp = torch.arange(0, n * kk + 1, kk, dtype=torch.int64, device=dev)
    p = torch.empty_like(dist)
    ctx.dev_affinities(rp, dist, n, perplexity, p)
    cap = 2 * n * kk
    orp = torch.empty(n + 1, dtype=torch.int64, device=dev)
    oc = torch.empty(cap, dtype=torch.int32, device=dev)
    ov = torch.empty(cap, dtype=torch.float64, device=dev)
    nnz = ctx.dev_joint(rp, idx, p, n, cap, orp, oc, ov)
    ctx.synchronize()
    host = dict(idx=idx.cpu().numpy(), dist=dist.cpu().numpy(), p=p.cpu().numpy(),
                P=(orp.cpu().numpy(), oc[:nnz].cpu().numpy(), ov[:nnz].cpu().numpy()))
    return host, (orp, oc[:nnz], ov[:nnz])


def run_schedule(ctx, Pd, n, c, params, snaps, seed=0, stop=None, steps=(), Y0=None):
    """The device optimizer over the real schedule; host copies of Y after the
    iterations in `snaps`, and for every t in `steps` the optimizer's whole
    state (Y, upd, gains; original order, via tsne_dev_opt_sync) before and
    after its own step t."""
    dev = Pd[0].device
    Yh, uh, gh = ctx.initWorkingSet(n, c, seed=seed)
    if Y0 is not None:
        Yh = Y0.copy()
    Y = torch.from_numpy(Yh).to(dev)
    u = torch.from_numpy(uh).to(dev)
    g = torch.from_numpy(gh).to(dev)
    ctx.dev_opt_setup(params, *Pd, n, Y, u, g)

    def state():
        ctx.dev_opt_sync()
        ctx.synchronize()
        return tuple(x.cpu().numpy().copy() for x in (Y, u, g))

    out, st = {}, {}
    for t in range(1, (stop or params.iterations) + 1):
        before = state() if t in steps else None
        ctx.dev_opt_step(t)
        if t in steps:
            st[t] = (before, state(), ctx.dev_opt_last_z())
        if t in snaps:
            ctx.dev_opt_sync()   # the caller's Y is written at sync (not by a step)
            ctx.synchronize()
            out[t] = Y.cpu().numpy().copy()
    return out, ctx.dev_opt_losses(), st


def momentum(t, T_):
    return 0.5 if t <= min(T_, 20) else 0.8


def check_opt_step(ctx, P, before, after, Z, t, T_, theta, metric, r0, nr, c=2, loss_gpu=None, lr=1000.0,
                   all_rows=True, key="step"):
    """The optimizer's OWN iteration t (attract_tiles / attract_rows, the
    Z-free loss terms, combine_update, centring -- tsne_dev_opt_step) against
    the oracle from the same state: TsneHelpers.scala:269-317 (gradient),
    :341-369 (updateEmbedding), :320-329 (centerEmbedding).
      * every row's attraction: the step's gradient (recovered from its
        momentum update) + F / Z, F the device BH of the same state, against
        the oracle's attraction over all of P, within 1e-6 of the row's scale
        (a dropped or doubled P entry anywhere fails it);
      * the step's gradient of rows [r0, r0+nr), recovered exactly from its
        momentum update u' = mom u - lr gain' grad, within 1e-4 x max|grad|
        (north_star) of the oracle's attraction + BH repulsion with the same Z;
      * the gains (the reference's sign rule; a sign may differ only where
        |grad| is inside the tolerance);
      * the new Y: Y' + mean = the oracle's uncentred update, i.e. the offset
        is one vector over the rows, and Y' is centred;
      * the loss of iteration t (t % 10 == 0) against the oracle's KL over
        every row of P with the same Z, at 1e-9.
    Z is the step's own BH normaliser (tsne_dev_opt_last_z); it must equal the
    sum of the per-point z of the same state (tsne_repulsion, whose sampled
    rows are checked against the oracle) to the two builds' near-exact bounds."""
    Y0, u0, g0 = before
    Y1, u1, g1 = after
    n = Y0.shape[0]
    ex, mom = exaggeration(t, T_), momentum(t, T_)
    F, z = ctx.repulsion(Y0, theta)
    assert abs(z.sum() - Z) <= (near_tol(ctx) + near_tol(ctx, ex == 1.0)) * Z, (t, "Z", Z, z.sum())
    # every row: the step's attraction (its gradient + F / Z, F the device BH of
    # the same state) against the oracle's attraction over the whole of P
    attr = O.attraction_rows if c == 2 else O.attraction3_rows
    if all_rows:
        a_o, _ = attr(*P, Y0, np.zeros((n, c)), Z, 0, n, metric=metric, exaggeration=ex)
        a_opt = (mom * u0 - u1) / (lr * g1) + F / Z
        scale = np.abs(a_o).sum(1) + np.abs(F / Z).sum(1) + 1e-300
        rel = np.abs(a_opt - a_o).sum(1) / scale
        bad = np.argsort(rel)[-5:][::-1]
        assert rel.max() <= 1e-6, (t, "attraction rows", [(int(i), float(rel[i]), int(P[0][i + 1] - P[0][i]),
                                                           a_opt[i].tolist(), a_o[i].tolist()) for i in bad])
    Q = np.ascontiguousarray(Y0[r0:r0 + nr])
    rep_o, z_o = (O.repulsion_queries if c == 2 else O.repulsion3_queries)(Y0, theta, Q, threads=THREADS)
    assert np.abs(z[r0:r0 + nr] - z_o).max() <= near_tol(ctx) * z_o.max(), (t, "per-point z")
    rep = np.zeros((n, c))
    rep[r0:r0 + nr] = rep_o
    g_o, _ = attr(*P, Y0, rep, Z, r0, r0 + nr, metric=metric, exaggeration=ex)
    rows = slice(r0, r0 + nr)
    tol = 1e-4 * np.abs(g_o).max()
    grad = (mom * u0[rows] - u1[rows]) / (lr * g1[rows])
    assert np.abs(grad - g_o).max() <= tol, (t, np.abs(grad - g_o).max(), tol)
    rel = row_relative(grad, g_o, "%s step t=%d" % (key, t))
    assert rel <= 1e-4, (t, "per-row relative gradient", rel)
    Yn, un, gn = (x[rows].copy() for x in (Y0, u0, g0))   # O.update works in place: copies, not views
    O.update(np.ascontiguousarray(g_o), Yn, un, gn, 0.01, mom, lr)
    assert ((gn == g1[rows]) | (np.abs(g_o) <= tol)).all(), (t, "gains")
    off = Yn - Y1[rows]
    spread = np.abs(off - off.mean(0)).max()
    assert spread <= 2.0 * lr * g1[rows].max() * tol + 1e-12 * np.abs(Yn).max(), (t, spread)
    assert np.abs(Y1.mean(0)).max() <= 1e-9 * np.abs(Y1).max(), (t, "centred")
    if loss_gpu is not None:
        _, l_o = attr(*P, Y0, np.zeros((n, c)), Z, 0, n, metric=metric, exaggeration=ex, want_loss=True)
        if not abs(loss_gpu - l_o) <= 1e-9 * abs(l_o):   # diagnostics: the attract_rows loss, the sum of P
            _, Zg, l_rows = ctx.gradient(*P, Y0, theta, metric, exaggeration=ex, want_loss=True)
            info = dict(t=t, loss_opt=loss_gpu, loss_oracle=l_o, loss_attract_rows=l_rows, Zopt=Z,
                        Zrep=z.sum(), Zgrad=Zg, sumP=float(P[2].sum()))
            if metric == "sqeuclidean" and c == 2:   # an independent numpy restatement, exact sum
                rp, cl, pv = P
                rows = np.repeat(np.arange(n), np.diff(rp))
                d = Y0[rows] - Y0[cl]
                q = 1.0 / (1.0 + (d * d).sum(1))
                pij = pv * ex
                terms = pij * np.log(pij / (q / Z))
                info.update(loss_numpy=math.fsum(terms), self_pairs=int((rows == cl).sum()),
                            nonpos=int((pv <= 0).sum()), nonfinite=int((~np.isfinite(terms)).sum()),
                            max_term=float(np.abs(terms).max()), nnz=len(pv))
            assert False, repr(info)


def full_config(ctx, Xd, X_host, k, metric, perplexity, theta, T_, c, snaps, grad_rows, q0, stop=None, steps=(),
                name="config"):
    n = Xd.shape[0]
    host, Pd = pipeline(ctx, Xd, k, metric, perplexity)
    check_knn_rows(X_host, host["idx"], host["dist"], k, metric, q0)
    rows = np.arange(q0, q0 + 64)
    check_affinity_rows(host["dist"], host["p"], perplexity, rows)
    check_joint_rows(host["idx"], host["p"], *host["P"], rows[:16])
    del host["idx"], host["dist"], host["p"]
    params = default_params(iterations=T_, theta=theta, metric=metric, n_components=c)
    Ys, losses, st = run_schedule(ctx, Pd, n, c, params, set(snaps), stop=stop, steps=set(steps))
    for t, nr in snaps.items():
        r0 = grad_rows
        check_gradient_snapshot(ctx, host["P"], Ys[t], theta, exaggeration(t + 1, T_), metric, r0, nr, c=c,
                                loss=(t == max(snaps)), key="%s snapshot t=%d" % (name, t))
    for t in sorted(steps):   # the optimizer's own step at config size
        check_opt_step(ctx, host["P"], *st[t], t, T_, theta, metric, grad_rows + 64, 64, c=c,
                       loss_gpu=losses.get(t), key=name)
    return losses


# ------------------------------------------------------------------- C1
def parse_loss_file(text):
    return {int(k): float(v) for k, v in re.findall(r"(\d+)=([-+0-9.eE]+|NaN)", text)}


def test_c1_cli_end_to_end_matches_oracle(ctx, tmp_path):
    """configs[0]: the reference's CPU-runnable case, through the native CLI
    with Tsne.main's flags and file formats."""
    X = CF.c1()
    n, d = X.shape
    (tmp_path / "in.csv").write_text(CF.to_coo_lines(X))
    r = subprocess.run([str(CLI), "--input", "in.csv", "--output", "out.csv", "--dimension", str(d),
                        "--knnMethod", "bruteforce", "--metric", "sqeuclidean", "--perplexity", "30",
                        "--iterations", "300", "--loss", "loss.txt"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    out = np.array([[float(v) for v in l.split(",")] for l in (tmp_path / "out.csv").read_text().splitlines()])
    assert np.array_equal(out[:, 0], np.arange(n))
    lg = parse_loss_file((tmp_path / "loss.txt").read_text())
    # the oracle pipeline from the same Y0 (the CLI's --randomState 0 stream)
    oi, od = O.knn(X, 90, threads=THREADS)
    rp = np.arange(0, n * 90 + 1, 90, dtype=np.int64)
    po, _ = O.affinities(rp, od.ravel(), 30.0)
    P = O.joint(rp, oi.ravel(), po, n)
    Y0, _, _ = ctx.initWorkingSet(n, 2, seed=0)
    runs = []
    for s in range(8):
        Yo = Y0 * (1 + (0.0 if s == 0 else 1e-15) * np.random.default_rng(s).normal(size=Y0.shape))
        runs.append(O.optimize(*P, Yo, np.zeros_like(Y0), np.ones_like(Y0), learning_rate=1000.0, iterations=300,
                               theta=0.25, threads=THREADS))
    lo = runs[0]
    assert sorted(lg) == sorted(lo) == list(range(10, 301, 10))
    for t in (10, 20, 30, 40, 50):
        assert abs(lg[t] - lo[t]) <= 0.01 * abs(lo[t]), (t, lg[t], lo[t])
    final = np.array([r_[300] for r_ in runs])
    mu, sd = final.mean(), final.std()
    assert abs(lg[300] - mu) <= 4.0 * sd + 0.01 * abs(mu), (lg[300], final)


def test_c1_library_stages_match_oracle(ctx):
    X = CF.c1()
    n = X.shape[0]
    gi, gd = ctx.kNearestNeighbors(X, 90)
    oi, od = O.knn(X, 90, threads=THREADS)
    assert np.array_equal(gi, oi) and np.array_equal(gd, od)
    rp = np.arange(0, n * 90 + 1, 90, dtype=np.int64)
    p = ctx.pairwiseAffinities(rp, gd.ravel(), 30.0)
    po, _ = O.affinities(rp, od.ravel(), 30.0)
    assert np.abs(p - po).max() <= 1e-12
    a = ctx.jointDistribution(rp, gi.ravel(), p, n)
    b = O.joint(rp, oi.ravel(), po, n)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and np.abs(a[2] - b[2]).max() <= 1e-15


# ------------------------------------------------------------------- C2
def test_c2_mnist_shaped_full_size(ctx):
    X = CF.c2()
    Xd = torch.from_numpy(X).cuda()
    losses = full_config(ctx, Xd, X, 90, "sqeuclidean", 30.0, 0.5, 1000, 2,
                         snaps={1: 32, 100: 64, 300: 64, 1000: 64}, grad_rows=40_000, q0=12_345,
                         steps=(300, 1000), name="C2")
    assert sorted(losses) == list(range(10, 1001, 10))
    assert all(np.isfinite(v) for v in losses.values())


# ------------------------------------------------------------------- C3
def test_c3_gmm_1m_full_size(ctx):
    Xd = CF.c3_torch()
    X = Xd.cpu().numpy()
    losses = full_config(ctx, Xd, X, 90, "sqeuclidean", 30.0, 0.5, 1000, 2,
                         snaps={1: 16, 200: 64, 400: 64, 1000: 64}, grad_rows=654_321, q0=123_456,
                         steps=(1, 200, 400, 1000), name="C3")
    assert sorted(losses) == list(range(10, 1001, 10))
    assert all(np.isfinite(v) for v in losses.values())


# ------------------------------------------------------------------- C4
def test_c4_sparse_cosine_3d_full_size(ctx):
    X = CF.c4()
    Xd = torch.from_numpy(X).cuda()
    # the whole schedule (round 6: past t = 300), the optimizer's own step
    # checked in the late phase too (t = 650, 1000)
    losses = full_config(ctx, Xd, X, 90, "cosine", 30.0, 0.5, 1000, 3, snaps={1: 16, 150: 32, 1000: 32},
                         grad_rows=250_000, q0=77_777, steps=(1, 120, 150, 300, 650, 1000), name="C4")
    assert sorted(losses) == list(range(10, 1001, 10))
    assert all(np.isfinite(v) for v in losses.values())


# ------------------------------------------------------------------- C5
def test_c5_cli_distance_matrix_end_to_end(ctx, tmp_path):
    """--inputDistanceMatrix through the native CLI (2,000 points, every
    off-diagonal pair and, second pass, the diagonal too)."""
    n = 2000
    for diag in (False, True):
        rp, col, d = CF.c5_matrix(n, diagonal=diag)
        rows = np.repeat(np.arange(n), np.diff(rp))
        (tmp_path / "dm.csv").write_text("".join(f"{a},{b},{c!r}\n" for a, b, c in
                                                 zip(rows.tolist(), col.tolist(), d.tolist())))
        r = subprocess.run([str(CLI), "--input", "dm.csv", "--output", "out.csv", "--dimension", "64",
                            "--knnMethod", "bruteforce", "--inputDistanceMatrix", "--perplexity", "30",
                            "--iterations", "60", "--theta", "0.5", "--loss", "loss.txt"], cwd=tmp_path,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        Yc = np.array([[float(v) for v in l.split(",")[1:]] for l in (tmp_path / "out.csv").read_text().splitlines()])
        lc = parse_loss_file((tmp_path / "loss.txt").read_text())
        po, _ = O.affinities(rp, d, 30.0)
        P = O.joint(rp, col, po, n)
        Y0, _, _ = ctx.initWorkingSet(n, 2, seed=0)
        Yo = Y0.copy()
        lo = O.optimize(*P, Yo, np.zeros_like(Y0), np.ones_like(Y0), iterations=60, theta=0.5, threads=THREADS)
        assert sorted(lc) == sorted(lo)
        assert [np.isnan(lc[t]) for t in sorted(lc)] == [np.isnan(lo[t]) for t in sorted(lo)]
        S = CF.support(P)
        _, _, kl_c = ctx.gradient(*S, Yc, 0.5, want_loss=True)
        _, _, kl_o = ctx.gradient(*S, Yo, 0.5, want_loss=True)
        assert abs(kl_c - kl_o) <= 0.01 * abs(kl_o), (diag, kl_c, kl_o)


def test_c5_distance_matrix_5k_matches_oracle(ctx):
    n = 5000
    rp, col, d = CF.c5_matrix(n)
    p = ctx.pairwiseAffinities(rp, d, 30.0)            # workgroup-per-row beta search
    po, _ = O.affinities(rp, d, 30.0)
    assert np.abs(p - po).max() <= 1e-12
    a = ctx.jointDistribution(rp, col, p, n)            # sorted, all mutual: no sort passes
    P = O.joint(rp, col, po, n)
    assert np.array_equal(a[0], P[0]) and np.array_equal(a[1], P[1]) and np.abs(a[2] - P[2]).max() <= 1e-15
    assert (P[2] == 0).any()                           # underflowed affinities: the reference's KL is NaN
    S = CF.support(P)
    Y0, _, _ = ctx.initWorkingSet(n, 2, seed=4)
    T_ = 60
    prm = default_params(iterations=T_, theta=0.5)
    snaps = {1, 30, 60}
    dev = torch.device("cuda", 0)
    Pd = tuple(torch.from_numpy(np.ascontiguousarray(x)).to(dev) for x in P)
    Y = torch.from_numpy(Y0.copy()).to(dev)
    u = torch.zeros_like(Y)
    g = torch.ones_like(Y)
    ctx.dev_opt_setup(prm, *Pd, n, Y, u, g)
    for t in range(1, T_ + 1):
        ctx.dev_opt_step(t)
        if t in snaps:   # per-iteration gradient parity at the trajectory's own states
            ctx.dev_opt_sync()
            ctx.synchronize()
            Yt = Y.cpu().numpy()
            ex = exaggeration(t + 1, T_)
            gg, Zg, Lg = ctx.gradient(*P, Yt, 0.5, exaggeration=ex, want_loss=True)
            r = O.gradient(*P, Yt, 0.5, exaggeration=ex, want_loss=True, threads=THREADS)
            assert np.abs(gg - r["grad"]).max() <= 1e-4 * np.abs(r["grad"]).max(), t
            assert abs(Zg - r["Z"]) <= near_tol(ctx) * r["Z"], t
            assert np.isnan(Lg) and np.isnan(r["loss"])
            _, _, kg = ctx.gradient(*S, Yt, 0.5, exaggeration=ex, want_loss=True)
            ro = O.gradient(*S, Yt, 0.5, exaggeration=ex, want_loss=True, threads=THREADS)
            assert abs(kg - ro["loss"]) <= 1e-9 * abs(ro["loss"]), t
    lg = ctx.dev_opt_losses()
    Yo = Y0.copy()
    lo = O.optimize(*P, Yo, np.zeros_like(Y0), np.ones_like(Y0), iterations=T_, theta=0.5, threads=THREADS)
    assert sorted(lg) == sorted(lo) == list(range(10, T_ + 1, 10))
    assert all(np.isnan(lg[t]) and np.isnan(lo[t]) for t in lg)
    _, _, kg = ctx.gradient(*S, Y.cpu().numpy(), 0.5, want_loss=True)
    _, _, ko = ctx.gradient(*S, Yo, 0.5, want_loss=True)
    assert abs(kg - ko) <= 0.01 * abs(ko), (kg, ko)


def test_c5_distance_matrix_50k_full_size(ctx):
    """C5 at its stated size (BASELINE configs[4]): the full 50,000 x 49,999
    sqeuclidean matrix of a 64-D GMM (2.5e9 entries, built on the device like
    bench.py --config c5) through affinities, joint and the device optimizer.
    Sampled affinity rows at 1e-12 and joint rows (pattern exact, values
    1e-13 relative) against the oracle / a restatement of jointDistribution;
    the optimizer's own step at t = 1 and t = 60 (check_opt_step: gradient
    rows at 1e-4 x max|grad|, gains, centred update); the loss keys with the
    reference's NaN (0 ln 0 of underflowed affinities, TsneHelpers.scala:300)."""
    n, d, T_ = 50_000, 64, 60
    m = n - 1
    dev = torch.device("cuda", 0)
    Xd = torch.from_numpy(CF.c5_points(n, d, 4)).to(dev)
    sq = (Xd * Xd).sum(1)
    dist = torch.empty((n, m), dtype=torch.float64, device=dev)
    col = torch.empty((n, m), dtype=torch.int32, device=dev)
    ar = torch.arange(n, device=dev, dtype=torch.int32)
    for b0 in range(0, n, 1024):
        b1 = min(n, b0 + 1024)
        D = (sq[b0:b1, None] + sq[None, :] - 2.0 * (Xd[b0:b1] @ Xd.T)).clamp_(min=0.0)
        keep = torch.ones((b1 - b0, n), dtype=torch.bool, device=dev)
        keep[torch.arange(b1 - b0, device=dev), torch.arange(b0, b1, device=dev)] = False
        dist[b0:b1] = D[keep].view(b1 - b0, m)
        col[b0:b1] = ar.expand(b1 - b0, n)[keep].view(b1 - b0, m)
        del D, keep
    rp = torch.arange(0, n * m + 1, m, dtype=torch.int64, device=dev)
    p = torch.empty_like(dist)
    ctx.dev_affinities(rp, dist, n, 30.0, p)
    ctx.synchronize()
    sample = [0, 1, 12_345, 31_337, n - 1]
    for i in sample:   # workgroup-per-row beta search over 49,999 entries
        po, _ = O.affinities(np.array([0, m], dtype=np.int64), dist[i].cpu().numpy(), 30.0)
        assert np.abs(p[i].cpu().numpy() - po).max() <= 1e-12, i
    # the host-buffer entry point (what the JNI bodies call) with all 2.5e9
    # entries: 64-bit counts and offsets end to end, the same values
    ph = ctx.pairwiseAffinities(rp.cpu().numpy(), dist.cpu().numpy().ravel(), 30.0)
    assert ph.size == n * m > 2 ** 31
    assert np.array_equal(ph, p.cpu().numpy().ravel())
    del ph, dist
    cap = n * m
    orp = torch.empty(n + 1, dtype=torch.int64, device=dev)
    oc = torch.empty(cap, dtype=torch.int32, device=dev)
    ov = torch.empty(cap, dtype=torch.float64, device=dev)
    nnz = ctx.dev_joint(rp, col, p, n, cap, orp, oc, ov)
    assert nnz == n * m
    tot = 2.0 * p.sum().item()
    jrows = torch.arange(n, device=dev)
    for i in sample[:3]:   # P_ij = (p_j|i + p_i|j) / sum J over the union (all mutual here)
        others = jrows[jrows != i]
        pos = torch.where(others > i, torch.full_like(others, i), torch.full_like(others, i - 1))
        want = ((p[i] + p[others, pos]) / tot).cpu().numpy()
        a, b = int(orp[i].item()), int(orp[i + 1].item())
        assert np.array_equal(oc[a:b].cpu().numpy(), others.cpu().numpy().astype(np.int32)), i
        got = ov[a:b].cpu().numpy()
        assert np.all(np.abs(got - want) <= 1e-13 * want + 2e-323), i   # + a few subnormal ulps
    underflow = bool((ov == 0).any().item())
    del col, p
    torch.cuda.empty_cache()
    Pd = (orp, oc, ov)
    params = default_params(iterations=T_, theta=0.5)
    r0, nr = 20_000, 32
    _, losses, st = run_schedule(ctx, Pd, n, 2, params, set(), seed=4, steps={1, 60})
    # the sampled rows of P on the host (the oracle's attraction reads rows [r0, r0 + nr) only)
    a, b = int(orp[r0].item()), int(orp[r0 + nr].item())
    rps = np.clip(orp.cpu().numpy() - a, 0, b - a)
    Ps = (rps, oc[a:b].cpu().numpy(), ov[a:b].cpu().numpy())
    for t in (1, 60):
        check_opt_step(ctx, Ps, *st[t], t, T_, 0.5, "sqeuclidean", r0, nr, all_rows=False, key="C5")
    assert sorted(losses) == list(range(10, T_ + 1, 10))
    assert all(np.isnan(losses[t]) == underflow for t in losses)
    del Pd, orp, oc, ov
    torch.cuda.empty_cache()
