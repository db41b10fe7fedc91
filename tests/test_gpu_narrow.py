"""The narrow layout of heavy BH groups (bhtree.hip "Narrow layout"): a
64-query group whose previous traversal cost >= Options::narrow x the mean
runs as 16 waves of 4 queries, lanes = (stack entry, query, child).  It opens
and summarises the same cells as the 64-query layout (QuadTree.scala:123-152)
and sums the same leaves and tiles; only the association of the sums
differs (and, for a query with more than 128 moment-eligible tiles, which of
them take moments: each <= mom_tol = 1e-12 relative).  So it must equal the
64-query layout to ~1e-12 and the oracle to the library's near-exact bound,
and be deterministic (fixed xor-butterfly reduction, no atomics on sums)."""
import numpy as np
import pytest
import torch

import oracle_ctypes as O
import tsne_amd as T
from tsne_amd.api import default_params

pytestmark = pytest.mark.gpu


def clustered(n, seed):
    """A mid-schedule-like embedding: 20 blobs of extent ~1 over a ~30-wide
    field, a quarter of each blob in a dense core (the heavy groups)."""
    rng = np.random.default_rng(seed)
    centres = rng.uniform(-15, 15, size=(20, 2))
    lab = rng.integers(0, 20, n)
    sd = np.where(rng.random(n) < 0.25, 0.02, 0.5)[:, None]
    return centres[lab] + rng.normal(size=(n, 2)) * sd


def layouts(Y, theta, factor):
    """(F, z) of the 64-query layout, then of the narrow one at `factor` (the
    selection runs at the end of a traversal, from its costs, for the next
    one: the first call with the option on only selects), and the number of
    narrow groups."""
    with T.Context(0) as c:
        c.set_option("reuse_costs", 1)
        c.set_option("narrow", 0)
        F0, z0 = c.repulsion(Y, theta)
        assert c.counter("bh.narrow_groups") == 0
        c.set_option("narrow", factor)
        Fw, zw = c.repulsion(Y, theta)
        assert c.counter("bh.narrow_groups") == 0
        # the same 64-query layout (block order from the recorded costs: re-association only)
        assert np.all(np.abs(zw - z0) <= 1e-12 * z0) and np.abs(Fw - F0).max() <= 1e-12 * np.abs(F0).max()
        F1, z1 = c.repulsion(Y, theta)
        ng = c.counter("bh.narrow_groups")
        F2, z2 = c.repulsion(Y, theta)   # the same selection (same costs): the same bits
        assert c.counter("bh.narrow_groups") == ng
    assert np.array_equal(F1, F2) and np.array_equal(z1, z2)
    return (F0, z0), (F1, z1), ng


@pytest.mark.parametrize("factor", [0.25, 3.0])
def test_narrow_repulsion_equals_wide(factor):
    """factor 0.25: the heavy-slot capacity (1/8 of the groups) fills;
    3: the library default, the dense cores only (if any group qualifies)."""
    n = 40_000
    Y = clustered(n, 5)
    (F0, z0), (F1, z1), ng = layouts(Y, 0.5, factor)
    assert ng > 0 or factor > 1
    assert np.all(np.abs(z1 - z0) <= 1e-11 * z0)
    assert np.abs(F1 - F0).max() <= 1e-11 * np.abs(F0).max()
    q = np.arange(0, n, 97)
    rep, zi = O.repulsion_queries(Y, 0.5, np.ascontiguousarray(Y[q]), threads=8)
    with T.Context(0) as c:
        tol = c.get_option("near_tol_early")
    assert np.abs(z1[q] - zi).max() <= tol * zi.max()
    assert np.abs(F1[q] - rep).max() <= tol * np.abs(rep).max()


def test_narrow_with_duplicates_and_ties():
    """Exact duplicates (the reference's multiplicities, virtual chain tops,
    key-tie groups) inside heavy groups, theta 0.25, against the oracle."""
    n = 20_000
    Y = clustered(n, 9)
    Y[[5, 900, 17_000]] = Y[5]
    Y[100:140] = Y[100]
    (F0, z0), (F1, z1), ng = layouts(Y, 0.25, 0.25)
    assert ng > 0
    assert np.all(np.abs(z1 - z0) <= 1e-11 * z0)
    assert np.abs(F1 - F0).max() <= 1e-11 * np.abs(F0).max()
    rep, zi = O.repulsion(Y, 0.25, threads=8)
    with T.Context(0) as c:
        tol = c.get_option("near_tol_early")
    assert np.abs(z1 - zi).max() <= tol * zi.max()
    assert np.abs(F1 - rep).max() <= tol * np.abs(rep).max()


def test_single_calls_are_history_free():
    """By default (reuse_costs 0) a single call is a function of its input:
    the same call twice gives the same bits whatever ran before."""
    Y = clustered(20_000, 7)
    with T.Context(0) as c:
        F0, z0 = c.repulsion(Y, 0.5)
        c.repulsion(Y * 1.5, 0.5)
        F1, z1 = c.repulsion(Y, 0.5)
        assert c.counter("bh.narrow_groups") == 0
    assert np.array_equal(F0, F1) and np.array_equal(z0, z1)


def test_narrow_small_embedding_moments():
    """The near-exact regime (tiles with moments) under the narrow layout:
    a 20k embedding of extent 0.03 with a dense core."""
    n = 20_000
    rng = np.random.default_rng(12)
    Y = rng.normal(size=(n, 2)) * 0.03
    Y[: n // 4] *= 0.01
    (F0, z0), (F1, z1), ng = layouts(Y, 0.5, 0.5)
    assert np.all(np.abs(z1 - z0) <= 1e-11 * z0)
    assert np.abs(F1 - F0).max() <= 1e-11 * np.abs(F0).max()
    rep, zi = O.repulsion(Y, 0.5, threads=8)
    with T.Context(0) as c:
        tol = c.get_option("near_tol_early")
    assert np.abs(z1 - zi).max() <= tol * zi.max()
    assert np.abs(F1 - rep).max() <= tol * np.abs(rep).max()


def test_optimizer_narrow_deterministic_and_equal():
    """The device optimizer with the narrow layout forced wide (factor 0.25):
    run twice -> bit-identical; against narrow off -> the same trajectory to
    re-association level over 150 iterations (the exaggerated phase and 49
    late ones)."""
    from test_gpu_parity import random_problem
    n = 6000
    rp, col, val = random_problem(n, 30, seed=23)
    Y0 = np.random.default_rng(4).normal(size=(n, 2)) * 1e-4
    p = default_params(iterations=150, theta=0.5)
    dev = torch.device("cuda", 0)
    Pd = tuple(torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (rp, col, val))

    def run(factor):
        with T.Context(0) as c:
            c.set_option("narrow", factor)
            Y = torch.from_numpy(Y0.copy()).to(dev)
            u, g = torch.zeros_like(Y), torch.ones_like(Y)
            c.dev_opt_setup(p, *Pd, n, Y, u, g)
            used = 0
            for t in range(1, p.iterations + 1):
                c.dev_opt_step(t)
                if t % 10 == 0:
                    used += c.counter("opt.narrow_groups")
            c.dev_opt_sync()
            c.synchronize()
            return Y.cpu().numpy(), c.dev_opt_losses(), used

    Ya, la, ua = run(0.25)
    Yb, lb, ub = run(0.25)
    assert ua > 0 and ua == ub
    assert np.array_equal(Ya, Yb) and la == lb
    Yc, lc, uc = run(0)
    assert uc == 0 and sorted(la) == sorted(lc)
    assert np.abs(Ya - Yc).max() <= 1e-6 * np.abs(Yc).max()
    for t in lc:
        assert abs(la[t] - lc[t]) <= 1e-7 * abs(lc[t]), t


@pytest.mark.parametrize("n,scale,theta", [(3000, 1e-4, 0.5), (20000, 0.02, 0.5), (20000, 3.0, 0.5),
                                           (20000, 0.1, 0.25), (600, 1.0, 0.0)])
def test_octal_records_match_binary_walk_and_oracle(n, scale, theta):
    """3-D: the octal-record traversals (8 queries x 8 children per wave, and
    64 queries per wave: "oct_records" 1 / 2) and the binary-node walk (0)
    against the octree restatement (oracle_gradient3): the same summarised
    cells; tiles are taken at real cells only by the records, within the
    near-exact bound.  The two record layouts take the same decisions: equal
    to re-association level."""
    from test_gpu_parity import random_problem
    rp, col, val = random_problem(n, 10, seed=n + int(scale * 100))
    Y = np.random.default_rng(n).normal(size=(n, 3)) * scale
    r = O.gradient3(rp, col, val, Y, theta, exaggeration=4.0, want_loss=True)
    F_o, z_o = r["rep"], r["zi"]
    tol = 1e-12 if theta == 0.0 else 1e-6
    out = {}
    for rec in (1, 2, 0):
        with T.Context(0) as c:
            c.set_option("oct_records", rec)
            c.set_option("oct_layout_switch", 0)   # each layout at every scale
            g, Z, loss = c.gradient(rp, col, val, Y, theta, exaggeration=4.0, want_loss=True)
            F, z = c.repulsion(Y, theta)
        assert np.abs(g - r["grad"]).max() <= tol * np.abs(r["grad"]).max(), rec
        assert abs(Z - r["Z"]) <= 1e-7 * r["Z"], rec
        assert np.abs(z - z_o).max() <= 1e-7 * z_o.max(), rec
        assert np.abs(F - F_o).max() <= 1e-6 * np.abs(F_o).max(), rec
        out[rec] = (F, z)
    assert np.abs(out[1][1] - out[0][1]).max() <= 2e-7 * out[0][1].max()
    assert np.abs(out[1][1] - out[2][1]).max() <= 1e-12 * out[1][1].max()
    assert np.abs(out[1][0] - out[2][0]).max() <= 1e-12 * np.abs(out[1][0]).max()
