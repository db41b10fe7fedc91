"""Tile streaming (bhtree.hip "Tile streaming", option "tile_stream"): the
traversal waves hand their finished tile lists to a persistent consumer grid
running beside the traversal on a stream of its own, instead of every list
waiting for the whole grid.  A list goes to whichever path claims it first,
and a consumer sums it exactly as the slot path (tile_apply -> moment_apply
-> chunk_combine) sums a one-chunk wave, so the bits do not depend on which
path took it or when.  With tile_stream_max below the chunking unit (4095) F
and z are the bits of no streaming; with the default threshold (the previous
plan's chunk unit) a handed-over list the plan would have chunked is one
chunk, a re-association.  The sums are those of the reference's walk either
way (QuadTree.scala:123-152)."""
import numpy as np
import pytest
import torch

import oracle_ctypes as O
import tsne_amd as T
from tsne_amd.api import default_params
from test_gpu_narrow import clustered

pytestmark = pytest.mark.gpu


def run(Y, theta, opts, calls=2):
    """(F, z) of the last of `calls` repulsion calls (the first selects the
    narrow groups and sets the streaming threshold of the next) and the lists
    the consumers summed."""
    with T.Context(0) as c:
        for k, v in opts.items():
            c.set_option(k, v)
        for _ in range(calls):
            F, z = c.repulsion(Y, theta)
        return F, z, c.counter("bh.stream_lists")


@pytest.mark.parametrize("blocks", [1, 2, 8])
@pytest.mark.parametrize("narrow", [0, 3])
def test_stream_bit_identical(blocks, narrow):
    """40k clustered points (dense cores: long lists, heavy waves), with and
    without the narrow layout, lists up to the chunking unit handed over: the
    same bits as the slot path."""
    Y = clustered(40_000, 5)
    F0, z0, l0 = run(Y, 0.5, {"narrow": narrow})
    F1, z1, l1 = run(Y, 0.5, {"narrow": narrow, "tile_stream": blocks, "tile_stream_max": 4095,
                                  "tile_stream_wait": 20000})
    assert l0 == 0 and l1 > 0
    assert np.array_equal(F1, F0) and np.array_equal(z1, z0)


@pytest.mark.parametrize("frac", [1.0, 4.0])
def test_stream_default_threshold(frac):
    """The default threshold (tile_stream_frac x the previous plan's chunk
    unit, set by the first call): deterministic, equal to no streaming to
    re-association."""
    Y = clustered(40_000, 6)
    F0, z0, _ = run(Y, 0.5, {"narrow": 0}, calls=3)
    # (consumers wait up to ~8 ms for a list: small inputs finish walks late relative to their start)
    opts = {"narrow": 0, "tile_stream": 2, "tile_stream_frac": frac, "tile_stream_wait": 20000}
    F1, z1, l1 = run(Y, 0.5, opts, calls=3)
    F2, z2, _ = run(Y, 0.5, opts, calls=3)
    assert l1 > 0
    assert np.array_equal(F1, F2) and np.array_equal(z1, z2)
    assert np.all(np.abs(z1 - z0) <= 1e-12 * z0)
    assert np.abs(F1 - F0).max() <= 1e-12 * np.abs(F0).max()


def test_stream_every_list_and_oracle():
    """tile_stream_max raised: every list handed over, the heavy ones one
    chunk (re-association only), against the oracle at the near-exact bound;
    twice the same bits."""
    n = 30_000
    Y = clustered(n, 8)
    Y[[5, 900, 17_000]] = Y[5]          # duplicates and a key-tie group inside lists
    Y[100:140] = Y[100]
    F0, z0, _ = run(Y, 0.25, {"narrow": 0})
    opts = {"narrow": 0, "tile_stream": 1, "tile_stream_max": 1 << 30, "tile_stream_wait": 20000}
    F1, z1, l1 = run(Y, 0.25, opts)
    F2, z2, _ = run(Y, 0.25, opts)
    assert l1 > 0
    assert np.array_equal(F1, F2) and np.array_equal(z1, z2)
    assert np.all(np.abs(z1 - z0) <= 1e-12 * z0)
    assert np.abs(F1 - F0).max() <= 1e-12 * np.abs(F0).max()
    q = np.arange(0, n, 53)
    rep, zi = O.repulsion_queries(Y, 0.25, np.ascontiguousarray(Y[q]), threads=8)
    with T.Context(0) as c:
        tol = c.get_option("near_tol_early")
    assert np.abs(z1[q] - zi).max() <= tol * zi.max()
    assert np.abs(F1[q] - rep).max() <= tol * np.abs(rep).max()


@pytest.mark.parametrize("n", [700, 6_001])
def test_stream_small_and_ragged(n):
    """Few waves (more consumers than lists) and a partial last group; the
    near-exact regime (moment lists) on a small embedding."""
    rng = np.random.default_rng(n)
    Y = rng.normal(size=(n, 2)) * 0.05
    Y[: n // 3] *= 0.01
    F0, z0, _ = run(Y, 0.5, {"root_tile": 0})
    F1, z1, _ = run(Y, 0.5, {"root_tile": 0, "tile_stream": 4, "tile_stream_max": 4095})
    assert np.array_equal(F1, F0) and np.array_equal(z1, z0)


def test_optimizer_stream():
    """The device optimizer over 150 iterations (exaggerated phase and 49 late
    ones) with streaming: lists up to the chunking unit -> the same trajectory
    and losses to the last bit; the default threshold -> twice the same bits,
    and the trajectory of no streaming to re-association level."""
    from test_gpu_parity import random_problem
    n = 6000
    rp, col, val = random_problem(n, 30, seed=23)
    Y0 = np.random.default_rng(4).normal(size=(n, 2)) * 1e-4
    p = default_params(iterations=150, theta=0.5)
    dev = torch.device("cuda", 0)
    Pd = tuple(torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (rp, col, val))

    def go(o):
        with T.Context(0) as c:
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
            return Y.cpu().numpy(), c.dev_opt_losses(), c.counter("opt.stream_lists")

    Ya, la, sa = go({})
    Yb, lb, sb = go({"tile_stream": 2, "tile_stream_max": 4095})
    assert sa == 0 and sb > 0
    assert np.array_equal(Ya, Yb) and la == lb
    Yc, lc, sc = go({"tile_stream": 2})
    Yd, ld, _ = go({"tile_stream": 2})
    assert sc > 0
    assert np.array_equal(Yc, Yd) and lc == ld
    assert np.abs(Yc - Ya).max() <= 1e-6 * np.abs(Ya).max()
    for t in la:
        assert abs(lc[t] - la[t]) <= 1e-7 * abs(la[t]), t


@pytest.mark.parametrize("front", [0.5, 1.0, 2.0])
def test_trav_front_order_bit_identical(front):
    """trav_front: the 64-query workgroups dispatched heavy-first (the order
    made with the narrow selection from the previous call's costs): every wave
    sums its own queries, so F and z keep their bits."""
    Y = clustered(40_000, 7)
    base = {"reuse_costs": 1}
    F0, z0, _ = run(Y, 0.5, base, calls=3)
    F1, z1, _ = run(Y, 0.5, dict(base, trav_front=front), calls=3)
    assert np.array_equal(F1, F0) and np.array_equal(z1, z0)


@pytest.mark.parametrize("front", [0.8, 1.5])
def test_trav_front_cur_bit_identical(front):
    """trav_front_cur: the dispatch order predicted from the points' previous
    costs through this build's Morton order (made on the second stream during
    the build): F and z keep their bits, single calls and the optimizer."""
    Y = clustered(40_000, 9)
    base = {"reuse_costs": 1}
    F0, z0, _ = run(Y, 0.5, base, calls=3)
    F1, z1, _ = run(Y, 0.5, dict(base, trav_front_cur=front), calls=3)
    assert np.array_equal(F1, F0) and np.array_equal(z1, z0)
    from test_gpu_parity import random_problem
    n = 6000
    rp, col, val = random_problem(n, 30, seed=29)
    Y0 = np.random.default_rng(5).normal(size=(n, 2)) * 1e-4
    p = default_params(iterations=150, theta=0.5)
    dev = torch.device("cuda", 0)
    Pd = tuple(torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (rp, col, val))

    def go(o):
        with T.Context(0) as c:
            c.set_option("root_tile", 0)
            for k, v in o.items():
                c.set_option(k, v)
            Yd = torch.from_numpy(Y0.copy()).to(dev)
            u, g = torch.zeros_like(Yd), torch.ones_like(Yd)
            c.dev_opt_setup(p, *Pd, n, Yd, u, g)
            for t in range(1, p.iterations + 1):
                c.dev_opt_step(t)
            c.dev_opt_sync()
            c.synchronize()
            return Yd.cpu().numpy(), c.dev_opt_losses()

    Ya, la = go({})
    Yb, lb = go({"trav_front_cur": front})
    assert np.array_equal(Ya, Yb) and la == lb
