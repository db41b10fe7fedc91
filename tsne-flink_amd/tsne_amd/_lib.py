"""ctypes declarations for libtsne_hip.so (include/tsne_hip.h)."""
import ctypes as C
import os
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent      # tsne-flink_amd/
METRICS = {"sqeuclidean": 0, "euclidean": 1, "cosine": 2}
UNIQUE_ID_BYTES = 128

STATUS = {0: "TSNE_OK", -1: "TSNE_ERR_ARG", -2: "TSNE_ERR_HIP", -3: "TSNE_ERR_NOMEM",
          -4: "TSNE_ERR_UNSUPPORTED", -5: "TSNE_ERR_CAPACITY", -6: "TSNE_ERR_COMM",
          -7: "TSNE_ERR_NO_DEVICE"}


class TsneError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"{STATUS.get(status, status)}: {msg}")
        self.status = status


class Params(C.Structure):
    _fields_ = [("n_components", C.c_int32), ("metric", C.c_int32), ("learning_rate", C.c_double),
                ("iterations", C.c_int32), ("early_exaggeration", C.c_double),
                ("initial_momentum", C.c_double), ("final_momentum", C.c_double),
                ("theta", C.c_double), ("min_gain", C.c_double)]


class CommOps(C.Structure):
    """tsne_comm_ops: host-buffer collectives supplied by the caller."""
    _fields_ = [("allreduce_sum_f64", C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_int64)),
                ("allreduce_sum_u64", C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.c_int64)),
                ("allgatherv", C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.POINTER(C.c_int64)))]


P = C.c_void_p
I32, I64, D, U64 = C.c_int32, C.c_int64, C.c_double, C.c_uint64
PI32, PI64, PD = C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_double)

# name -> (restype, argtypes); every symbol include/tsne_hip.h declares.
SIGNATURES = {
    "tsne_abi_version": (C.c_int, []),
    "tsne_last_error": (C.c_char_p, []),
    "tsne_params_default": (None, [C.POINTER(Params)]),
    "tsne_metric_from_name": (C.c_int, [C.c_char_p, PI32]),
    "tsne_shard_rows": (C.c_int, [I64, I32, I32, PI64, PI64]),
    "tsne_coo_to_csr": (C.c_int, [P, P, P, I64, I64, P, P, P]),
    "tsne_balance_cuts": (C.c_int, [P, I64, I64, I32, I32, P]),
    "tsne_dev_balance_cuts": (C.c_int, [P, P, I64, I32, P]),
    "tsne_ctx_create": (C.c_int, [I32, C.POINTER(P)]),
    "tsne_ctx_create_multi": (C.c_int, [P, I32, C.POINTER(P)]),
    "tsne_ctx_destroy": (C.c_int, [P]),
    "tsne_ctx_set_stream": (C.c_int, [P, P]),
    "tsne_ctx_stream": (P, [P]),
    "tsne_ctx_synchronize": (C.c_int, [P]),
    "tsne_comm_unique_id": (C.c_int, [C.c_char_p]),
    "tsne_ctx_init_comm": (C.c_int, [P, I32, I32, C.c_char_p]),
    "tsne_ctx_rank": (C.c_int, [P, PI32, PI32]),
    "tsne_ctx_init_comm_callbacks": (C.c_int, [P, I32, I32, P, P]),
    "tsne_knn": (C.c_int, [P, P, I64, I32, I32, I32, I64, I64, P, P]),
    "tsne_pairwise_affinities": (C.c_int, [P, P, P, I64, D, P]),
    "tsne_project_knn": (C.c_int, [P, P, I64, I32, I32, I32, I32, P, P, P]),
    "tsne_dev_project_knn": (C.c_int, [P, P, I64, I32, I32, I32, I32, P, P, P]),
    "tsne_joint_distribution": (C.c_int, [P, P, P, P, I64, I64, P, P, P, PI64]),
    "tsne_gradient": (C.c_int, [P, P, P, P, I64, P, I32, D, D, P, PD, PD]),
    "tsne_gradient_c": (C.c_int, [P, P, P, P, I64, I32, P, I32, D, D, P, PD, PD]),
    "tsne_update_embedding": (C.c_int, [P, I64, I32, P, P, P, P, D, D, D]),
    "tsne_repulsion": (C.c_int, [P, P, I64, I32, D, P, P]),
    "tsne_dev_repulsion": (C.c_int, [P, P, I64, I32, D, P, P]),
    "tsne_center_embedding": (C.c_int, [P, I64, I32, P]),
    "tsne_init_working_set": (C.c_int, [P, I64, I32, U64, P, P, P]),
    "tsne_optimize": (C.c_int, [P, C.POINTER(Params), P, P, P, I64, P, P, P, P, P, I32, PI32]),
    "tsne_dev_knn": (C.c_int, [P, P, I64, I32, I32, I32, I64, I64, P, P]),
    "tsne_dev_pairwise_affinities": (C.c_int, [P, P, P, I64, D, P]),
    "tsne_dev_joint_distribution": (C.c_int, [P, P, P, P, I64, I64, P, P, P, PI64]),
    "tsne_dev_opt_setup": (C.c_int, [P, C.POINTER(Params), P, P, P, I64, P, P, P]),
    "tsne_dev_opt_step": (C.c_int, [P, I32]),
    "tsne_dev_opt_sync": (C.c_int, [P]),
    "tsne_dev_opt_losses": (C.c_int, [P, P, P, I32, PI32]),
    "tsne_dev_opt_profile": (C.c_int, [P, I32, P, P]),
    "tsne_dev_opt_last_z": (C.c_int, [P, PD]),
    "tsne_dev_opt_attract_log": (C.c_int, [P, P, P, P, I32, PI32]),
    "tsne_ctx_stage_ms": (C.c_int, [P, C.c_char_p, P, I32, PI32]),
    "tsne_ctx_set_option": (C.c_int, [P, C.c_char_p, D]),
    "tsne_ctx_get_option": (C.c_int, [P, C.c_char_p, PD]),
    "tsne_hip_versions": (C.c_int, [PI32, PI32]),
    "tsne_ctx_counter": (C.c_int, [P, C.c_char_p, PI64]),
    "tsne_debug_wave_log": (C.c_int, [P, P, I64, PI64]),
    "tsne_ctx_loop_profile": (C.c_int, [P, C.c_char_p, I64, PI64]),
}

_lib = None


def lib_path():
    # TSNE_HIP_LIB: another build of the same library (A/B experiments)
    return Path(os.environ["TSNE_HIP_LIB"]) if os.environ.get("TSNE_HIP_LIB") else PKG_ROOT / "libtsne_hip.so"


def lib():
    """Load libtsne_hip.so from the package tree; raise if it was not built."""
    global _lib
    if _lib is None:
        path = lib_path()
        if not path.exists():
            raise TsneError(-2, f"{path} not built (run `make -C {PKG_ROOT}`); no CPU fallback exists")
        # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64
        # (same soname as /opt/rocm's).  Loaded first, it is the one this
        # library binds to; if this library initialised /opt/rocm's runtime
        # first, torch's own would later find no GPU ("No HIP GPUs are
        # available", measured on the GPU box).  So torch, when present, goes
        # first (TSNE_NO_TORCH_PRELOAD=1: not; a broken torch install only
        # skips the preload).  The runtime that was loaded must then be of the
        # major version the library was built against (checked below).
        if not os.environ.get("TSNE_NO_TORCH_PRELOAD"):
            try:
                import torch  # noqa: F401
            except Exception:  # noqa: BLE001 -- any failure: load without it
                pass
        L = C.CDLL(str(path))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        built, rt = C.c_int32(), C.c_int32()
        if L.tsne_hip_versions(C.byref(built), C.byref(rt)) == 0 and rt.value // 10**7 != built.value // 10**7:
            raise TsneError(-2, f"{path} was built for HIP {built.value} but the process loaded HIP runtime "
                                f"{rt.value} (major versions differ)")
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        raise TsneError(rc, lib().tsne_last_error().decode(errors="replace"))
    return rc


def metric_from_name(name):
    """Tsne.getMetric (Tsne.scala:161-168)."""
    out = C.c_int32()
    check(lib().tsne_metric_from_name(name.encode(), C.byref(out)))
    return out.value


def shard_rows(n, world, rank):
    a, b = C.c_int64(), C.c_int64()
    check(lib().tsne_shard_rows(n, world, rank, C.byref(a), C.byref(b)))
    return a.value, b.value


def balance_cuts(bcost, n, world, bucket=256):
    """tsne_balance_cuts: cost-balanced query cuts (host mirror of the device rule)."""
    import numpy as np
    b = np.ascontiguousarray(bcost, dtype=np.uint64)
    out = np.zeros(world + 1, dtype=np.int64)
    check(lib().tsne_balance_cuts(b.ctypes.data_as(C.c_void_p), b.size, n, world, bucket,
                                  out.ctypes.data_as(C.c_void_p)))
    return out
