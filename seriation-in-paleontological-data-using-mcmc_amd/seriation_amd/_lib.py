"""ctypes binding of libseriation.so (the C ABI declared in include/seriation.h).

The library is built in-tree (``make -C seriation-in-paleontological-data-using-mcmc_amd``
or ``__graft_entry__.build()``).  There is deliberately no Python or CPU fallback for the
sweep: if the library or a gfx950 device is missing, calls fail loudly.
"""
import ctypes
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("SERIATION_LIB") or os.path.join(PKG_DIR, "build", "libseriation.so")

SR_OK = 0
SR_EINVAL = -1
SR_EPARSE = -2
SR_EHEADER = -3
SR_ENOMEM = -4
SR_EDEVICE = -5
SR_EUNSUPPORTED = -6
SR_EIO = -7
SR_EINCONSISTENT = -8
SR_MAXS = 2000
SR_F_NO_CHECK = 1
SR_F_HBM_COLUMNS = 2
SR_F_LDS_COLUMNS = 4
SR_F_DEBUG_CHECK = 8
SR_F_DEBUG_PRINT = 16
SR_F_RNG_PHILOX = 32
SR_F_DIAG = 64
SR_F_GENERIC_KERNEL = 128


class SrError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        msg = _lib().sr_strerror(code).decode() if _LIB is not None else str(code)
        super().__init__("%s%s (code %d)" % (what + ": " if what else "", msg, code))


class sr_dataset(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int32), ("M", ctypes.c_int32), ("nh", ctypes.c_int32),
                ("X", ctypes.POINTER(ctypes.c_uint8)), ("hard", ctypes.POINTER(ctypes.c_uint8))]


class sr_chain_spec(ctypes.Structure):
    _fields_ = [("chain_id", ctypes.c_int32), ("seed", ctypes.c_uint64)]


class sr_run_opts(ctypes.Structure):
    _fields_ = [("burnin_calls", ctypes.c_int32), ("sample_calls", ctypes.c_int32),
                ("sweeps_per_call", ctypes.c_int32), ("manycd", ctypes.c_int32),
                ("device", ctypes.c_int32), ("block_threads", ctypes.c_int32),
                ("calls_per_launch", ctypes.c_int32), ("flags", ctypes.c_int32)]


class sr_chain_summary(ctypes.Structure):
    _fields_ = [("chain_id", ctypes.c_int32), ("consistent", ctypes.c_int32),
                ("exp_loglik", ctypes.c_double), ("exp_c", ctypes.c_double), ("exp_d", ctypes.c_double)]


class sr_record(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int32), ("M", ctypes.c_int32),
                ("a", ctypes.POINTER(ctypes.c_int32)), ("b", ctypes.POINTER(ctypes.c_int32)),
                ("pi", ctypes.POINTER(ctypes.c_int32)),
                ("c", ctypes.c_double), ("d", ctypes.c_double), ("loglik", ctypes.c_double),
                ("cv", ctypes.POINTER(ctypes.c_double)), ("dv", ctypes.POINTER(ctypes.c_double))]


class sr_posterior_out(ctypes.Structure):
    _fields_ = [("pair_order", ctypes.POINTER(ctypes.c_double)), ("alive", ctypes.POINTER(ctypes.c_double)),
                ("false_alive", ctypes.POINTER(ctypes.c_double)), ("false_ones", ctypes.POINTER(ctypes.c_double)),
                ("exp_pi", ctypes.POINTER(ctypes.c_double)), ("exp_a", ctypes.POINTER(ctypes.c_double)),
                ("kernel_ms", ctypes.c_double)]


SINK_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32,
                           ctypes.POINTER(sr_record))

# every symbol include/seriation.h declares (tests/test_abi.py checks the export list)
PUBLIC_SYMBOLS = [
    "sr_parse_dataset", "sr_load_dataset", "sr_free_dataset", "sr_save_dataset_bin", "sr_load_dataset_bin",
    "sr_default_opts", "sr_rng_env_setup",
    "sr_run_chains", "sr_run_to_dirs", "sr_run_chains_multi", "sr_run_to_dirs_multi", "sr_session_create", "sr_session_set_stream",
    "sr_session_run", "sr_session_sync", "sr_session_records", "sr_session_record_capacity",
    "sr_session_fetch_records", "sr_session_reset_records", "sr_session_fetch_chain_records", "sr_session_copy_chain_records", "sr_session_summaries",
    "sr_session_fetch_cd_vectors", "sr_session_manycd", "sr_session_state_cd",
    "sr_session_state",
    "sr_session_accept_counts", "sr_session_fallback_counts", "sr_session_debug_flagged", "sr_session_last_kernel_ms", "sr_session_block_threads", "sr_session_variant", "sr_session_specialized",
    "sr_session_checkpoint", "sr_session_restore",
    "sr_session_destroy", "sr_specialize", "sr_posterior", "sr_session_posterior", "sr_strerror", "sr_device_count", "sr_version",
]

_LIB = None


def _lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise ImportError("libseriation.so not built (%s); run __graft_entry__.build()" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    c_int, c_i32, c_void_p, c_double = ctypes.c_int, ctypes.c_int32, ctypes.c_void_p, ctypes.c_double
    sig = {
        "sr_parse_dataset": (c_int, [ctypes.c_char_p, ctypes.c_size_t, c_i32, P(sr_dataset)]),
        "sr_load_dataset": (c_int, [ctypes.c_char_p, c_i32, P(sr_dataset)]),
        "sr_free_dataset": (None, [P(sr_dataset)]),
        "sr_save_dataset_bin": (c_int, [P(sr_dataset), ctypes.c_char_p]),
        "sr_load_dataset_bin": (c_int, [ctypes.c_char_p, P(sr_dataset)]),
        "sr_default_opts": (None, [P(sr_run_opts)]),
        "sr_rng_env_setup": (c_int, [P(ctypes.c_uint64), c_i32]),
        "sr_run_chains": (c_int, [P(sr_dataset), P(sr_chain_spec), c_i32, P(sr_run_opts), SINK_FN,
                                  c_void_p, P(sr_chain_summary)]),
        "sr_run_to_dirs": (c_int, [P(sr_dataset), P(sr_chain_spec), c_i32, P(sr_run_opts),
                                   ctypes.c_char_p, P(sr_chain_summary)]),
        "sr_run_chains_multi": (c_int, [P(sr_dataset), P(sr_chain_spec), c_i32, P(sr_run_opts), P(c_i32), c_i32,
                                        SINK_FN, c_void_p, P(sr_chain_summary)]),
        "sr_run_to_dirs_multi": (c_int, [P(sr_dataset), P(sr_chain_spec), c_i32, P(sr_run_opts), P(c_i32), c_i32,
                                         ctypes.c_char_p, P(sr_chain_summary)]),
        "sr_session_create": (c_int, [P(sr_dataset), P(sr_chain_spec), c_i32, P(sr_run_opts), P(c_void_p)]),
        "sr_session_set_stream": (c_int, [c_void_p, c_void_p]),
        "sr_session_run": (c_int, [c_void_p, c_i32, c_i32]),
        "sr_session_sync": (c_int, [c_void_p]),
        "sr_session_records": (c_i32, [c_void_p]),
        "sr_session_record_capacity": (c_i32, [c_void_p]),
        "sr_session_fetch_records": (c_int, [c_void_p, c_i32, c_i32, P(ctypes.c_int16), P(c_double)]),
        "sr_session_reset_records": (c_int, [c_void_p]),
        "sr_session_fetch_chain_records": (c_int, [c_void_p, c_i32, c_i32, c_i32, P(ctypes.c_int16), P(c_double)]),
        "sr_session_copy_chain_records": (c_int, [c_void_p, c_i32, c_i32, c_i32, c_void_p, c_void_p]),
        "sr_session_summaries": (c_int, [c_void_p, c_i32, c_i32, P(sr_chain_summary)]),
        "sr_session_fetch_cd_vectors": (c_int, [c_void_p, c_i32, c_i32, P(c_double)]),
        "sr_session_manycd": (c_i32, [c_void_p]),
        "sr_session_state_cd": (c_int, [c_void_p, c_i32, P(c_double), P(c_double)]),
        "sr_session_state": (c_int, [c_void_p, c_i32, P(c_i32), P(c_i32), P(c_i32), P(c_double), P(c_i32)]),
        "sr_session_accept_counts": (c_int, [c_void_p, c_i32, P(ctypes.c_int64)]),
        "sr_session_fallback_counts": (c_int, [c_void_p, c_i32, P(ctypes.c_int64)]),
        "sr_session_debug_flagged": (c_int, [c_void_p, c_i32]),
        "sr_session_last_kernel_ms": (c_double, [c_void_p]),
        "sr_session_block_threads": (c_i32, [c_void_p]),
        "sr_session_variant": (c_i32, [c_void_p]),
        "sr_session_specialized": (c_i32, [c_void_p]),
        "sr_session_checkpoint": (c_int, [c_void_p, ctypes.c_char_p]),
        "sr_session_restore": (c_int, [P(sr_dataset), ctypes.c_char_p, P(sr_run_opts), P(c_void_p)]),
        "sr_session_destroy": (None, [c_void_p]),
        "sr_specialize": (c_int, [P(sr_dataset), P(sr_run_opts)]),
        "sr_posterior": (c_int, [P(sr_dataset), P(ctypes.c_int16), c_i32, c_i32, c_i32, c_i32, P(sr_posterior_out)]),
        "sr_session_posterior": (c_int, [c_void_p, P(c_i32), c_i32, c_i32, c_i32, c_i32, P(sr_posterior_out)]),
        "sr_strerror": (ctypes.c_char_p, [c_int]),
        "sr_device_count": (c_int, []),
        "sr_version": (ctypes.c_char_p, []),
        # test hooks (not part of the public ABI)
        "sr_host_exp_log": (None, [P(c_double), ctypes.c_long, P(c_double), P(c_double)]),
        "sr_host_run_add": (c_double, [c_double, c_double, ctypes.c_long]),
        "sr_host_run_sub": (ctypes.c_long, [P(c_double), c_double, ctypes.c_long]),
        "sr_host_philox": (None, [P(ctypes.c_uint32), P(ctypes.c_uint32), P(ctypes.c_uint32)]),
        "sr_host_mt_untemper": (None, [P(ctypes.c_uint32), ctypes.c_long, P(ctypes.c_uint32), P(ctypes.c_uint32)]),
        "sr_host_initial_checkpoint": (c_int, [P(sr_dataset), P(sr_chain_spec), c_i32, ctypes.c_char_p]),
        "sr_host_init_chain": (c_int, [P(sr_dataset), ctypes.c_uint64, P(c_i32), P(c_i32), P(c_i32),
                                       P(c_double), P(ctypes.c_uint64)]),
        "sr_spec_cache_path": (c_int, [c_int, c_int, c_int, c_int, ctypes.c_char_p, ctypes.c_size_t]),
        "sr_session_debug_counters": (c_int, [c_void_p, P(ctypes.c_ulonglong)]),
        "sr_session_spec_embedded": (c_i32, [c_void_p]),
        "sr_spec_is_embedded": (c_int, [c_int, c_int, c_int, c_int]),
        "sr_device_selftest_math": (c_int, [c_int, P(c_double), ctypes.c_long, P(c_double), P(c_double)]),
    }
    for name, (res, args) in sig.items():
        if not hasattr(L, name):   # an older build (A/B variants); tests/test_abi.py checks the product's exports
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = L
    return L


def lib():
    return _lib()
