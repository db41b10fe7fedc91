"""Work splitting of long BH walks (bhtree.hip "Spill", option "spill"): a
64-query walk past its pop budget hands the rest of its stack -- (cell, lane
mask) entries -- to the next level's task list; the drain launches walk those
subtrees for the same 64 queries (splitting again past the task budget), and
the tasks' sums reach F and z through fixed-point accumulators.  Every cell is opened or
summarised exactly as in the unsplit walk (QuadTree.scala:123-152: the
decision depends on the query and the cell only), so the result equals the
unsplit traversal to re-association level and the oracle to the near-exact
bound.  The split points depend on pop counts alone and the fixed-point adds
are associative: the same input gives the same bits, whichever wave took
which task."""
import numpy as np
import pytest
import torch

import oracle_ctypes as O
import tsne_amd as T
from tsne_amd.api import default_params
from test_gpu_narrow import clustered

pytestmark = pytest.mark.gpu


def split_vs_whole(Y, theta, force, reps=2):
    """(F, z) unsplit, then with every walk split after `force` pops (twice:
    the same bits), and the number of tasks the split calls made."""
    with T.Context(0) as c:
        c.set_option("narrow", 0)
        F0, z0 = c.repulsion(Y, theta)
        assert c.counter("bh.spill_tasks") == 0
        c.set_option("spill_force", force)
        outs = [c.repulsion(Y, theta) for _ in range(reps)]
        tasks = c.counter("bh.spill_tasks")
        assert c.counter("bh.spill_flags") == 0
    for F, z in outs[1:]:
        assert np.array_equal(F, outs[0][0]) and np.array_equal(z, outs[0][1])
    return (F0, z0), outs[0], tasks


@pytest.mark.parametrize("force", [1, 6, 64])
def test_split_repulsion_equals_whole(force):
    """force 1: every walk splits at its first batch, tasks split again after
    one pop (thousands of tasks per group); 64: only the heavy walks split."""
    n = 40_000
    Y = clustered(n, 5)
    (F0, z0), (F1, z1), tasks = split_vs_whole(Y, 0.5, force)
    assert tasks > 0
    assert np.all(np.abs(z1 - z0) <= 1e-12 * z0)
    assert np.abs(F1 - F0).max() <= 1e-12 * np.abs(F0).max()
    q = np.arange(0, n, 97)
    rep, zi = O.repulsion_queries(Y, 0.5, np.ascontiguousarray(Y[q]), threads=8)
    with T.Context(0) as c:
        tol = c.get_option("near_tol_early")
    assert np.abs(z1[q] - zi).max() <= tol * zi.max()
    assert np.abs(F1[q] - rep).max() <= tol * np.abs(rep).max()


def test_split_with_duplicates_and_ties():
    """Exact duplicates (multiplicities, virtual chain tops, key-tie groups)
    inside split walks, theta 0.25, against the whole oracle."""
    n = 20_000
    Y = clustered(n, 9)
    Y[[5, 900, 17_000]] = Y[5]
    Y[100:140] = Y[100]
    (F0, z0), (F1, z1), tasks = split_vs_whole(Y, 0.25, 3)
    assert tasks > 0
    assert np.all(np.abs(z1 - z0) <= 1e-12 * z0)
    assert np.abs(F1 - F0).max() <= 1e-12 * np.abs(F0).max()
    rep, zi = O.repulsion(Y, 0.25, threads=8)
    with T.Context(0) as c:
        tol = c.get_option("near_tol_early")
    assert np.abs(z1 - zi).max() <= tol * zi.max()
    assert np.abs(F1 - rep).max() <= tol * np.abs(rep).max()


def test_split_small_embedding_moments():
    """The near-exact regime: the tasks' tile pages take subtree moments in
    place (tile_apply<true>), a 20k embedding of extent 0.03 with a dense core
    (root-tile mode off, so that the full tree and its tiles run)."""
    n = 20_000
    rng = np.random.default_rng(12)
    Y = rng.normal(size=(n, 2)) * 0.03
    Y[: n // 4] *= 0.01
    Y[n // 2:] += 0.5
    (F0, z0), (F1, z1), tasks = split_vs_whole(Y, 0.5, 2)
    assert tasks > 0
    assert np.all(np.abs(z1 - z0) <= 1e-11 * z0)
    assert np.abs(F1 - F0).max() <= 1e-11 * np.abs(F0).max()
    rep, zi = O.repulsion(Y, 0.5, threads=8)
    with T.Context(0) as c:
        tol = c.get_option("near_tol_early")
    assert np.abs(z1 - zi).max() <= tol * zi.max()
    assert np.abs(F1 - rep).max() <= tol * np.abs(rep).max()


def test_split_one_drain():
    """spill_drains 1: the traversal's own tasks are all taken by one
    no-split drain launch."""
    Y = clustered(20_000, 3)
    with T.Context(0) as c:
        c.set_option("narrow", 0)
        F0, z0 = c.repulsion(Y, 0.5)
        c.set_option("spill_force", 2)
        c.set_option("spill_drains", 1)
        F1, z1 = c.repulsion(Y, 0.5)
        assert c.counter("bh.spill_tasks") > 0 and c.counter("bh.spill_flags") == 0
    assert np.all(np.abs(z1 - z0) <= 1e-12 * z0)
    assert np.abs(F1 - F0).max() <= 1e-12 * np.abs(F0).max()


@pytest.mark.parametrize("opts", [{"spill": 1.0}, {"spill": 0.5, "spill_task": 0.1}, {"spill_force": 8}])
def test_optimizer_split_deterministic_and_equal(opts):
    """The device optimizer with split walks (budgets from the previous
    traversal's mean cost, or forced): twice -> bit-identical; against no
    splitting -> the same trajectory to re-association level over 150
    iterations (the exaggerated phase and 49 late ones)."""
    from test_gpu_parity import random_problem
    n = 6000
    rp, col, val = random_problem(n, 30, seed=23)
    Y0 = np.random.default_rng(4).normal(size=(n, 2)) * 1e-4
    p = default_params(iterations=150, theta=0.5)
    dev = torch.device("cuda", 0)
    Pd = tuple(torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (rp, col, val))

    def run(o):
        with T.Context(0) as c:
            c.set_option("narrow", 0)
            c.set_option("root_tile", 0)
            for k, v in o.items():
                c.set_option(k, v)
            Y = torch.from_numpy(Y0.copy()).to(dev)
            u, g = torch.zeros_like(Y), torch.ones_like(Y)
            c.dev_opt_setup(p, *Pd, n, Y, u, g)
            for t in range(1, p.iterations + 1):
                c.dev_opt_step(t)
            c.dev_opt_sync()
            c.synchronize()
            return Y.cpu().numpy(), c.dev_opt_losses(), c.counter("opt.spill_tasks"), c.counter("opt.spill_flags")

    Ya, la, ta, fa = run(opts)
    Yb, lb, tb, fb = run(opts)
    assert ta > 0 and ta == tb and fa == 0 and fb == 0
    assert np.array_equal(Ya, Yb) and la == lb
    Yc, lc, tc, _ = run({})
    assert tc == 0 and sorted(la) == sorted(lc)
    assert np.abs(Ya - Yc).max() <= 1e-6 * np.abs(Yc).max()
    for t in lc:
        assert abs(la[t] - lc[t]) <= 1e-7 * abs(lc[t]), t
