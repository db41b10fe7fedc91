"""Scheduling options of the 2-D optimizer that move kernels between streams
or change their grids without touching any sum: the trajectory must be
bit-identical to the default schedule's.

  attract_overlap 0  the non-loss attraction after the BH kernels instead of
                     beside them;
  attract_split x    the non-loss tiled attraction before the tree build on a
                     share x of the CUs (persistent workgroups, each row block
                     summed exactly as before)."""
import numpy as np
import pytest
import torch

import tsne_amd as T
from tsne_amd.api import default_params
from test_gpu_parity import random_problem

pytestmark = pytest.mark.gpu


def run(opts, n=60_000, iterations=60, seed=17):
    rp, col, val = random_problem(n, 20, seed=seed)
    Y0 = np.random.default_rng(seed).normal(size=(n, 2)) * 2.0   # past the root-tile phase from t = 1
    p = default_params(iterations=iterations, theta=0.5)
    dev = torch.device("cuda", 0)
    Pd = tuple(torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (rp, col, val))
    with T.Context(0) as c:
        for k, v in opts.items():
            c.set_option(k, v)
        Y = torch.from_numpy(Y0.copy()).to(dev)
        u, g = torch.zeros_like(Y), torch.ones_like(Y)
        c.dev_opt_setup(p, *Pd, n, Y, u, g)
        for t in range(1, p.iterations + 1):
            c.dev_opt_step(t)
        c.synchronize()
        return Y.cpu().numpy(), c.dev_opt_losses()


@pytest.mark.parametrize("opts", [{"attract_overlap": 0}, {"attract_split": 0.5}, {"attract_split": 0.1}])
def test_schedule_options_bit_identical(opts):
    Ya, la = run({})
    Yb, lb = run(opts)
    assert la == lb
    assert np.array_equal(Ya, Yb)
