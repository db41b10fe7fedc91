"""tsne_amd -- Python binding of libtsne_hip (the MI355X-native t-SNE hot path).

Thin ctypes layer over the C ABI in include/tsne_hip.h; used by the tests,
bench.py and __graft_entry__.  The library must be built in-tree
(`make -C tsne-flink_amd`); there is no CPU fallback: every call fails loudly
if the HIP library or a GPU is missing.
"""
from ._lib import (METRICS, TsneError, balance_cuts, lib, lib_path, metric_from_name,  # noqa: F401
                   shard_rows)
from .api import Context, Params, project_shifts  # noqa: F401
