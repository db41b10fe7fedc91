"""Synthetic inputs of BASELINE.json's configs (SURVEY.md 8d "Synthetic inputs").

The reference ships no generators; these are the build's own, seeded:
  C1  2,000 x 50, 5 centres ~ N(0, 10^2 I), points = centre + N(0, I), seed 0
  C2  70,000 x 784 MNIST-shaped: 10 centres in [0,1]^784 on a random ~20 %
      support, points = clip(centre + N(0, 0.15^2) on the support, 0, 1)
      quantised to k/255, seed 1
  C3  1,000,000 x 128 GMM: 10 centres ~ N(0, 5^2 I), within-blob N(0, I),
      rounded to fp32 (exact MFMA inputs), seed 2 (torch, on the device)
  C4  500,000 x 300 sparse: 20 non-negative topic profiles, each row draws 30
      distinct dimensions (10 % density) from its topic with log-normal
      magnitudes, seed 3
  C5  50,000-point GMM in 64-D (C3-style, seed 4) whose full sqeuclidean
      distance matrix (diagonal excluded) is the input
"""
import numpy as np


def c1(n=2000, d=50, seed=0):
    rng = np.random.default_rng(seed)
    centres = rng.normal(size=(5, d)) * 10.0
    return centres[rng.integers(0, 5, n)] + rng.normal(size=(n, d))


def c2(n=70_000, d=784, seed=1):
    rng = np.random.default_rng(seed)
    support = rng.random((10, d)) < 0.2
    centres = rng.random((10, d)) * support
    lab = rng.integers(0, 10, n)
    X = np.empty((n, d))
    for a in range(0, n, 10_000):      # chunks: bounded temporaries
        b = min(n, a + 10_000)
        noise = rng.normal(0.0, 0.15, (b - a, d)) * support[lab[a:b]]
        X[a:b] = np.round(np.clip(centres[lab[a:b]] + noise, 0.0, 1.0) * 255.0) / 255.0
    return X


def c3_torch(n=1_000_000, d=128, seed=2, device="cuda"):
    """The bench's C3 generator (bench.py gmm), on the device."""
    import torch
    g = torch.Generator(device=device).manual_seed(seed)
    centers = torch.randn(10, d, generator=g, device=device, dtype=torch.float64) * 5.0
    lab = torch.randint(0, 10, (n,), generator=g, device=device)
    X = centers[lab] + torch.randn(n, d, generator=g, device=device, dtype=torch.float64)
    return X.float().double().contiguous()


def c4(n=500_000, d=300, nnz_row=30, seed=3):
    """Dense n x d array holding the sparse rows (the COO triples are its nonzeros)."""
    rng = np.random.default_rng(seed)
    topics = rng.gamma(0.3, 1.0, (20, d)) + 1e-3
    topics /= topics.sum(1, keepdims=True)
    logp = np.log(topics)
    lab = rng.integers(0, 20, n)
    X = np.zeros((n, d))
    for a in range(0, n, 25_000):
        b = min(n, a + 25_000)
        keys = logp[lab[a:b]] + rng.gumbel(size=(b - a, d))      # Gumbel top-k: sampling without replacement
        cols = np.argpartition(-keys, nnz_row, axis=1)[:, :nnz_row]
        vals = rng.lognormal(0.0, 1.0, (b - a, nnz_row))
        np.put_along_axis(X[a:b], cols, vals, axis=1)
    return X


def c5_points(n=50_000, d=64, seed=4):
    rng = np.random.default_rng(seed)
    centres = rng.normal(size=(10, d)) * 5.0
    return (centres[rng.integers(0, 10, n)] + rng.normal(size=(n, d))).astype(np.float32).astype(np.float64)


def to_coo_lines(X):
    """Tsne.readInput's COO text (i,j,v per nonzero), Java double formatting not needed."""
    i, j = np.nonzero(X)
    v = X[i, j].tolist()
    return "".join(f"{a},{b},{c!r}\n" for a, b, c in zip(i.tolist(), j.tolist(), v))


def c5_matrix(n=5000, d=64, seed=4, diagonal=False):
    """C5's input as CSR rows in file order: row i = (i, j, sqeuclidean(x_i, x_j))
    for every j (j != i unless `diagonal`), as Tsne.readDistanceMatrix feeds
    them to the affinities (Tsne.scala:69-70, 155-159).  Distances from the
    norm expansion, clamped at 0 (any values do: they are the input)."""
    X = c5_points(n, d, seed)
    sq = (X * X).sum(1)
    D = np.maximum(sq[:, None] + sq[None, :] - 2.0 * (X @ X.T), 0.0)
    if diagonal:
        np.fill_diagonal(D, 0.0)
        col = np.tile(np.arange(n, dtype=np.int32), n)
        return np.arange(0, n * n + 1, n, dtype=np.int64), col, D.ravel()
    mask = ~np.eye(n, dtype=bool)
    col = np.nonzero(mask)[1].astype(np.int32)
    return np.arange(0, n * (n - 1) + 1, n - 1, dtype=np.int64), col, D[mask]


def support(P):
    """The entries of a CSR P with P_ij > 0 (the KL over them is finite)."""
    rp, col, val = P
    keep = val > 0.0
    rows = np.repeat(np.arange(len(rp) - 1), np.diff(rp))[keep]
    nrp = np.zeros(len(rp), dtype=np.int64)
    np.add.at(nrp, rows + 1, 1)
    return np.cumsum(nrp), col[keep], val[keep]
