"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports
every symbol include/tsne_hip.h declares, and its host-only logic (metric
names, shard arithmetic, error reporting) behaves like the reference."""
import re
from pathlib import Path

import pytest

import tsne_amd as T
from tsne_amd._lib import SIGNATURES

ROOT = Path(__file__).resolve().parent.parent


def declared_symbols():
    text = (ROOT / "include" / "tsne_hip.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(tsne_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported():
    L = T.lib()
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(SIGNATURES), set(syms) ^ set(SIGNATURES)


def test_abi_version():
    assert T.lib().tsne_abi_version() == 2


def test_hip_runtime_version_matches_build():
    """The HIP runtime the process loaded (torch's bundled one when torch is
    imported first) has the major version the library was built against
    (tsne_amd.lib() refuses it otherwise).  No device needed."""
    import ctypes as C
    b, r = C.c_int32(), C.c_int32()
    assert T.lib().tsne_hip_versions(C.byref(b), C.byref(r)) == 0
    assert b.value // 10 ** 7 == r.value // 10 ** 7 >= 6


@pytest.mark.parametrize("name,val", [("sqeuclidean", 0), ("euclidean", 1), ("cosine", 2)])
def test_metric_names(name, val):
    # Tsne.getMetric (Tsne.scala:161-168)
    assert T.metric_from_name(name) == val


def test_unknown_metric_is_illegal_argument():
    with pytest.raises(T.TsneError) as e:
        T.metric_from_name("manhattan")
    assert e.value.status == -1 and "not defined" in str(e.value)


@pytest.mark.parametrize("n,world", [(10, 3), (1_000_000, 8), (7, 8), (0, 2), (129, 2)])
def test_shard_rows_partition(n, world):
    got = [T.shard_rows(n, world, r) for r in range(world)]
    assert got[0][0] == 0 and got[-1][1] == n
    for (a, b), (c, d) in zip(got, got[1:]):
        assert b == c and a <= b
    chunk = -(-n // world)
    assert all(b - a <= chunk for a, b in got)


def test_default_params_match_reference_flags():
    # Tsne.scala:47-63 defaults; minGain TsneHelpers.scala:386
    from tsne_amd.api import default_params
    p = default_params()
    assert (p.n_components, p.metric, p.learning_rate, p.iterations) == (2, 0, 1000.0, 300)
    assert (p.early_exaggeration, p.initial_momentum, p.final_momentum) == (4.0, 0.5, 0.8)
    assert (p.theta, p.min_gain) == (0.25, 0.01)


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(T.TsneError) as e:
        T.Context(0)
    assert e.value.status == -7


def test_create_multi_argument_errors():
    """tsne_ctx_create_multi validates the device list before touching a GPU."""
    import ctypes as C
    import numpy as np
    L = T.lib()
    h = C.c_void_p()
    for devs in ([0, 0, 1], [1, 2, 1]):
        d = np.array(devs, dtype=np.int32)
        rc = L.tsne_ctx_create_multi(d.ctypes.data_as(C.c_void_p), len(devs), C.byref(h))
        assert rc == -1 and b"distinct" in L.tsne_last_error()
    rc = L.tsne_ctx_create_multi(None, 0, C.byref(h))
    assert rc == -1


def coo_to_csr(row, col, val, n):
    import ctypes as C
    import numpy as np
    row = np.ascontiguousarray(row, dtype=np.int32)
    col = np.ascontiguousarray(col, dtype=np.int32)
    val = None if val is None else np.ascontiguousarray(val, dtype=np.float64)
    rp = np.zeros(n + 1, dtype=np.int64)
    oc = np.zeros(max(1, len(col)), dtype=np.int32)
    ov = None if val is None else np.zeros(max(1, len(val)))
    p = lambda a: None if a is None else a.ctypes.data_as(C.c_void_p)
    rc = T.lib().tsne_coo_to_csr(p(row), p(col), p(val), len(row), n, p(rp), p(oc), p(ov))
    return rc, rp, oc[:len(col)], (None if ov is None else ov[:len(col)])


def test_coo_to_csr_groups_rows_stably():
    """tsne_coo_to_csr: the JNI bodies' groupBy(0) (TsneHelpers.scala:162-196)
    -- rows in index order, each row's entries in input order, empty rows kept."""
    import numpy as np
    rng = np.random.default_rng(5)
    n, nnz = 300, 5000
    row = rng.integers(0, n, nnz)
    row[row % 7 == 3] = 11            # a heavy row; some rows stay empty
    col = rng.integers(0, 10 ** 6, nnz)
    val = rng.random(nnz)
    rc, rp, oc, ov = coo_to_csr(row, col, val, n)
    assert rc == 0
    order = np.argsort(row, kind="stable")
    assert np.array_equal(rp, np.concatenate([[0], np.cumsum(np.bincount(row, minlength=n))]))
    assert np.array_equal(oc, col[order]) and np.array_equal(ov, val[order])
    rc, rp2, oc2, _ = coo_to_csr(row, col, None, n)
    assert rc == 0 and np.array_equal(rp2, rp) and np.array_equal(oc2, oc)
    rc, rp3, _, _ = coo_to_csr([], [], [], 4)
    assert rc == 0 and list(rp3) == [0, 0, 0, 0, 0]


def test_coo_to_csr_rejects_bad_rows():
    rc, _, _, _ = coo_to_csr([0, 5], [1, 2], [1.0, 2.0], 5)
    assert rc == -1 and b"out of [0, n)" in T.lib().tsne_last_error()
    rc, _, _, _ = coo_to_csr([0, -1], [1, 2], [1.0, 2.0], 5)
    assert rc == -1
