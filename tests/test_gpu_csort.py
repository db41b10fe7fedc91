"""The trees' Morton sort from the previous build's order (csort.hip): keys
ascending, ties by point index -- the same permutation as rocPRIM's stable
radix sort of (key, index), so every result downstream is bit-identical.
Checked through the device optimizer (a full build every iteration, 2-D and
3-D, with exact duplicates and key ties), against Options::coherent_sort = 0."""
import numpy as np
import pytest
import torch

import tsne_amd as T
from tsne_amd.api import default_params
from test_gpu_parity import random_problem

pytestmark = pytest.mark.gpu


def ring_problem(n, half=5):
    """A symmetric P without a kNN (sizes the oracle's O(n^2) kNN cannot reach):
    point i joined to i +- 1 .. i +- half (mod n), every entry 1 / (2 half n).
    (A ring's diameter is n / (2 half): run it with graph_order 0.)"""
    off = np.concatenate([np.arange(-half, 0), np.arange(1, half + 1)])
    col = np.sort((np.arange(n)[:, None] + off[None, :]) % n, axis=1).astype(np.int32).ravel()
    rp = np.arange(0, n * 2 * half + 1, 2 * half, dtype=np.int64)
    val = np.full(col.size, 1.0 / (2 * half * n))
    return rp, col, val


def run(n, C, coherent, seed, iterations=40, dups=False, scale=3.0, problem=None, options=()):
    rp, col, val = problem if problem is not None else random_problem(n, 20, seed=seed)
    Y0 = np.random.default_rng(seed).normal(size=(n, C)) * scale
    if dups:   # exact duplicates (the reference's multiplicities) and a key-tie run
        Y0[[3, 500, n - 7]] = Y0[3]
        Y0[1000:1040] = Y0[1000]
    p = default_params(iterations=iterations, theta=0.5, n_components=C)
    dev = torch.device("cuda", 0)
    Pd = tuple(torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (rp, col, val))
    with T.Context(0) as c:
        c.set_option("coherent_sort", coherent)
        for k, v in options:
            c.set_option(k, v)
        Y = torch.from_numpy(Y0.copy()).to(dev)
        u, g = torch.zeros_like(Y), torch.ones_like(Y)
        c.dev_opt_setup(p, *Pd, n, Y, u, g)
        over = 0
        for t in range(1, p.iterations + 1):
            c.dev_opt_step(t)
            if coherent and C == 2:
                over += c.counter("opt.csort_oversized")
        c.dev_opt_sync()
        c.synchronize()
        return Y.cpu().numpy(), c.dev_opt_losses(), over


@pytest.mark.parametrize("n,C,dups", [(50_000, 2, False), (50_000, 2, True), (40_000, 3, False), (40_000, 3, True)])
def test_coherent_sort_bit_identical(n, C, dups):
    Ya, la, over = run(n, C, 1, 31, dups=dups)
    Yb, lb, _ = run(n, C, 0, 31, dups=dups)
    assert over == 0   # oversampled splitters: every bucket within the LDS capacity
    assert la == lb
    assert np.array_equal(Ya, Yb)


def test_coherent_sort_at_the_largest_bucket_count():
    """n = 1.2M: 1024 buckets, 4096 splitter samples merged from 8 sorted runs
    of 512 (the run capacity exactly) -- rocPRIM's permutation every iteration."""
    n = 1_200_000
    prob = ring_problem(n)
    opts = (("graph_order", 0),)
    Ya, la, over = run(n, 2, 1, 5, iterations=4, problem=prob, options=opts)
    Yb, lb, _ = run(n, 2, 0, 5, iterations=4, problem=prob, options=opts)
    assert la == lb
    assert np.array_equal(Ya, Yb)


def test_coherent_sort_after_a_jump_and_oversized_buckets():
    """A large move between builds (half the embedding scaled x50 and shifted,
    half shrunk), then 12k copies of one point (equal keys: no splitter can
    cut them, the bucket exceeds the LDS capacity -> the global-memory path):
    rocPRIM's permutation every time, so the repulsion is bit-identical."""
    n = 60_000
    rng = np.random.default_rng(4)
    Y = rng.normal(size=(n, 2))
    Y2 = np.concatenate([Y[: n // 2] * 50.0 + 7.0, Y[n // 2:] * 0.01], axis=0)
    Y3 = Y2.copy()
    Y3[5000:17000] = Y3[5000]
    out = {}
    for cs in (1, 0):
        with T.Context(0) as c:
            c.set_option("coherent_sort", cs)
            c.repulsion(Y, 0.5)
            r2 = c.repulsion(Y2, 0.5)
            r3 = c.repulsion(Y3, 0.5)
            if cs:
                assert c.counter("bh.csort_oversized") >= 1
            out[cs] = (r2, r3)
    for k in range(2):
        assert np.array_equal(out[1][k][0], out[0][k][0]) and np.array_equal(out[1][k][1], out[0][k][1])
