"""Loaders for the committed reference fixtures (tests/golden/)."""
import json
from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden"


def goldens():
    return json.loads((GOLDEN / "reference_goldens.json").read_text())


def read_coo_dense(path, dimension):
    """Tsne.readInput (Tsne.scala:138-153): COO (i, j, v) -> dense rows.
    Returns (ids, X) with ids in ascending order."""
    rows = {}
    for line in Path(path).read_text().splitlines():
        if not line.strip():
            continue
        i, j, v = line.split(",")[:3]
        rows.setdefault(int(i), np.zeros(dimension))[int(j)] += float(v)
    ids = sorted(rows)
    return np.array(ids, dtype=np.int64), np.stack([rows[i] for i in ids])


def dense_input():
    return read_coo_dense(GOLDEN / "dense_input.csv", 28 * 28)


def triples_to_csr(triples, n):
    """(i, j, v) triples -> CSR with rows sorted by column."""
    t = sorted((int(a), int(b), float(c)) for a, b, c in triples)
    row_ptr = np.zeros(n + 1, dtype=np.int64)
    for a, _, _ in t:
        row_ptr[a + 1] += 1
    row_ptr = np.cumsum(row_ptr)
    col = np.array([b for _, b, _ in t], dtype=np.int32)
    val = np.array([c for _, _, c in t], dtype=np.float64)
    return row_ptr, col, val


def csr_to_dict(row_ptr, col, val):
    out = {}
    for i in range(len(row_ptr) - 1):
        for e in range(row_ptr[i], row_ptr[i + 1]):
            out[(i, int(col[e]))] = float(val[e])
    return out
