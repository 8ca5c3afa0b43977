"""ctypes binding of libskyline_hip.so (declared in include/skyline_hip.h).

The library is the product: every call below runs the gfx950 HIP path.  There is
no CPU fallback — if the library or a HIP device is missing, calls raise.

`torch` (when importable) is imported BEFORE the library is loaded: torch's wheel
ships its own libamdhip64.so (same soname), and loading torch first makes both
share one HIP runtime, so torch device pointers and library pointers mix freely.
"""
import ctypes
import os

try:  # single HIP runtime per process: torch's copy, if torch is present
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the binding itself
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("SKYLINE_HIP_LIB", os.path.join(PKG_DIR, "build", "libskyline_hip.so"))

SKY_OK = 0
SKY_E_ARG = -1
SKY_E_HIP = -2
SKY_E_CAPACITY = -3
SKY_E_NAN = -4
SKY_E_NOMEM = -5
SKY_E_NOLIB = -6
SKY_E_RETRY = -7

SKY_MAX_DIMS = 16
CSV_OK, CSV_MALFORMED, CSV_BAD_ID, CSV_ARITY = 0, 1, 2, 3

ALGO_DIM, ALGO_GRID, ALGO_ANGLE = 0, 1, 2
ALGOS = {"mr-dim": ALGO_DIM, "mr-grid": ALGO_GRID, "mr-angle": ALGO_ANGLE}
SEM_REFERENCE, SEM_COMPLETE = 0, 1
DIST_UNIFORM, DIST_CORRELATED, DIST_ANTI, DIST_STD_ANTI, DIST_MIXED = 0, 1, 2, 3, 4
DISTS = {"uniform": 0, "correlated": 1, "anti_correlated": 2, "std_anti": 3, "mixed": 4}
PHASES = ["pruners", "filter", "compact", "sort", "dedup", "local_sfs", "global_sfs", "fate"]

c_p = ctypes.c_void_p
c_i32 = ctypes.c_int32
c_i64 = ctypes.c_int64
c_int = ctypes.c_int
c_dbl = ctypes.c_double
P_i64 = ctypes.POINTER(ctypes.c_int64)
P_i32 = ctypes.POINTER(ctypes.c_int32)
P_dbl = ctypes.POINTER(ctypes.c_double)

# name -> (argtypes); every function returns int except the two string getters
SIGNATURES = {
    "sky_ctx_create": [P_i32, c_int, c_int, c_int, c_int, c_dbl, ctypes.POINTER(c_p)],
    "sky_ctx_destroy": [c_p],
    "sky_ctx_set_semantics": [c_p, c_int],
    "sky_ctx_set_stream": [c_p, c_p],
    "sky_ctx_set_grid_filter": [c_p, c_int],
    "sky_ctx_sync": [c_p],
    "sky_ctx_info": [c_p, P_i32, P_i32, P_i32],
    "sky_part_info": [c_p, P_i32, P_i32],
    "sky_stream_info": [c_p, P_i32],
    "sky_ctx_warmup": [c_p],
    "sky_ctx_wait_stream": [c_p, c_p],
    "sky_ctx_signal_stream": [c_p, c_p],
    "sky_partition_keys": [c_p, c_p, c_i64, c_p],
    "sky_partition_keys_dev": [c_p, c_p, c_i64, c_p],
    "sky_part_open": [c_p, c_i32, ctypes.POINTER(c_p)],
    "sky_part_close": [c_p],
    "sky_part_insert": [c_p, c_p, c_p, c_i64],
    "sky_parts_insert": [c_int, c_p, c_p, c_p, c_p],
    "sky_part_size": [c_p, P_i64],
    "sky_part_snapshot": [c_p, c_p, c_p, c_i64, P_i64],
    "sky_part_sizes": [c_p, P_i64, P_i64],
    "sky_part_snapshot_reps": [c_p, c_p, c_p, c_i64, c_p, c_p, c_i64, P_i64, P_i64],
    "sky_global_merge": [c_p, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, P_i64],
    "sky_parts_global_merge": [c_p, c_int, c_p, c_p, c_p, c_p, c_i64, P_i64],
    "sky_global_merge_reps": [c_p, c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, P_i64],
    "sky_global_stats": [c_p, c_p, c_p, P_i32],
    "sky_global_stats_set": [c_p, c_i32, c_p, c_p],
    "sky_query": [c_p, c_p, c_p, c_i64, c_p, c_p, c_i64, P_i64],
    "sky_query_dev": [c_p, c_p, c_p, c_i64, c_p, c_p, c_i64, P_i64],
    "sky_dist_export_dev": [c_p, c_p, c_p, c_i64, c_p, c_i64],
    "sky_dist_reblock_dev": [c_p, c_p, c_i64],
    "sky_dist_merge_dev": [c_p, c_p, c_i32, c_i32, c_i64, c_p, c_p, c_i64, c_p],
    "sky_dist_finish": [c_p, c_p, c_i64, P_i64, P_i64],
    "sky_profile_host_syncs": [c_p, P_i64],
    "sky_parse_csv_dev": [c_p, c_p, c_i64, c_p, c_p, c_i64, P_i64, P_i64, c_p],
    "sky_parse_csv": [c_p, c_p, c_i64, c_p, c_p, c_i64, P_i64, P_i64],
    "sky_format_csv_dev": [c_p, c_p, c_p, c_i64, c_p, c_i64, P_i64],
    "sky_stream_create": [c_p, c_i64, ctypes.POINTER(c_p)],
    "sky_stream_destroy": [c_p],
    "sky_stream_append": [c_p, c_p, c_p, c_i64],
    "sky_stream_append_dev": [c_p, c_p, c_p, c_i64],
    "sky_stream_size": [c_p, P_i64, P_i64],
    "sky_stream_vectors": [c_p, P_i64],
    "sky_stream_reserve": [c_p, c_i64],
    "sky_stream_query": [c_p, c_p, c_p, c_i64, P_i64],
    "sky_stream_query_dev": [c_p, c_p, c_p, c_i64, P_i64],
    "sky_stream_query_async": [c_p, c_p, c_p, c_i64, P_i64],
    "sky_stream_wait": [c_p, P_dbl],
    "sky_synth_dev": [c_p, c_int, c_int, c_int, ctypes.c_uint64, c_i64, c_i64, c_p, c_p],
    "sky_synth": [c_int, c_int, c_int, c_int, ctypes.c_uint64, c_i64, c_i64, c_p, c_p],
    "sky_dev_alloc": [c_p, c_i64, ctypes.POINTER(c_p)],
    "sky_dev_free": [c_p, c_p],
    "sky_memcpy_h2d": [c_p, c_p, c_p, c_i64],
    "sky_memcpy_d2h": [c_p, c_p, c_p, c_i64],
    "sky_profile_enable": [c_p, c_int],
    "sky_profile_phases": [c_p, c_p, c_p],
    "sky_profile_kernel": [c_p, ctypes.c_char_p, P_dbl, P_i64, P_i64],
    "sky_profile_dominance": [c_p, P_i64],
    "sky_profile_reset": [c_p],
    "sky_profile_sort_dev": [c_p, c_p, c_p, c_i64, P_i32, P_dbl],
    "sky_profile_pairs_dev": [c_p, c_p, c_p, c_i64, c_p, P_i32, P_dbl],
    "sky_last_error": [],
    "sky_version": [],
    "sky_device_count": [P_i32],
    "sky_device_for_subtask": [c_i32, c_i32, P_i32],
}


class SkylineError(RuntimeError):
    """Raised for a negative status; mirrors the RuntimeException a Java shim throws."""

    def __init__(self, code, msg):
        super().__init__(f"skyline_hip status {code}: {msg}")
        self.code = code


_lib = None


def lib():
    """Load (once) and return the library; raises OSError if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} not found: run `make -C flink-skyline-qos_amd` (or __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        for name, argt in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = ctypes.c_char_p if name in ("sky_last_error", "sky_version") else ctypes.c_int
        _lib = L
    return _lib


def check(rc):
    if rc != SKY_OK:
        raise SkylineError(rc, lib().sky_last_error().decode(errors="replace"))
    return rc


def exported_symbols_in_header(header_path=None):
    """Names of every entry point declared in include/skyline_hip.h."""
    import re
    header_path = header_path or os.path.join(os.path.dirname(PKG_DIR), "include", "skyline_hip.h")
    txt = open(header_path).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(sky_\w+)\s*\(", txt, re.M)))
