"""ctypes binding of libnrgpu.so (the C ABI declared in include/nrgpu.h).

The HIP library is the product: there is no CPU fallback. If the shared library is missing
this module raises at import time, and every data-plane call goes to the GPU.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.environ.get("NRGPU_LIB") or os.path.join(PKG_ROOT, "lib", "libnrgpu.so")  # env: A/B builds

# import torch first (when present) so that the process has ONE HIP runtime: torch ships
# its own libamdhip64.so.7 and the loader then reuses it for libnrgpu.so by SONAME.
try:  # pragma: no cover - depends on the image
    import torch  # noqa: F401
except Exception:  # noqa: BLE001
    torch = None

NRG_OK = 0
NRG_E_INVAL = -1
NRG_E_HIP = -2
NRG_E_TABLE_FULL = -3
NRG_E_RING_FULL = -4
NRG_E_NOMEM = -5
NRG_E_NOT_SYNCED = -6
NRG_E_CAPACITY = -7
NRG_E_NODEV = -8
NRG_E_COMM = -9
NRG_E_TIMEOUT = -10
NRG_GROUP_DEFAULT_TIMEOUT_MS = 300000
NRG_GROUP_ID_BYTES = 128
NRG_MAX_PARTS = 64

NRG_DS_HASHMAP = 1
NRG_DS_STACK = 2
NRG_DS_SYNTHETIC = 3

NRG_STACK_POP = 0
NRG_STACK_PUSH = 1
NRG_SYNTH_WRITE_ONLY = 0
NRG_SYNTH_READ_WRITE = 1


class NrgError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = _lib.nrg_strerror(code).decode() if _lib is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


class Config(C.Structure):
    _fields_ = [
        ("ds_kind", C.c_uint32),
        ("log2_slots", C.c_uint32),
        ("log_bytes", C.c_uint64),
        ("max_batch", C.c_uint64),
        ("max_reads", C.c_uint64),
        ("stack_capacity", C.c_uint64),
        ("synth_n", C.c_uint64),
        ("synth_cold_reads", C.c_uint32),
        ("synth_cold_writes", C.c_uint32),
        ("synth_hot_reads", C.c_uint32),
        ("synth_hot_writes", C.c_uint32),
        ("stack_push_resp", C.c_uint32),
        ("replica_id", C.c_uint32),
        ("pipeline", C.c_uint32),
    ]


class LogInfo(C.Structure):
    _fields_ = [
        ("size", C.c_uint64),
        ("head", C.c_uint64),
        ("tail", C.c_uint64),
        ("ctail", C.c_uint64),
        ("ltail", C.c_uint64),
        ("replica_id", C.c_uint32),
        ("ds_kind", C.c_uint32),
    ]


class Round(C.Structure):
    """nrg_round: one group member's part of a round (device pointers on its GPU)."""

    _fields_ = [
        ("recs", C.c_void_p),
        ("n", C.c_uint64),
        ("resp", C.c_void_p),
        ("some", C.c_void_p),
        ("get_keys", C.c_void_p),
        ("n_gets", C.c_uint64),
        ("get_vals", C.c_void_p),
        ("get_found", C.c_void_p),
    ]


vp = C.c_void_p
u64 = C.c_uint64
u32 = C.c_uint32
u64p = C.POINTER(C.c_uint64)

# every symbol declared in include/nrgpu.h, with its ctypes signature
SIGNATURES = {
    "nrg_config_default": (None, [C.POINTER(Config), u32]),
    "nrg_open": (C.c_int, [C.c_int, C.POINTER(Config), C.POINTER(vp)]),
    "nrg_close": (C.c_int, [vp]),
    "nrg_set_stream": (C.c_int, [vp, vp]),
    "nrg_get_stream": (vp, [vp]),
    "nrg_own_stream": (vp, [vp]),
    "nrg_sync": (C.c_int, [vp]),
    "nrg_join": (C.c_int, [vp]),
    "nrg_strerror": (C.c_char_p, [C.c_int]),
    "nrg_version": (C.c_char_p, []),
    "nrg_device_count": (C.c_int, []),
    "nrg_log_append": (C.c_int, [vp, vp, u64, u32, u64p]),
    "nrg_log_append_async": (C.c_int, [vp, vp, u64, u32, u64p]),
    "nrg_log_append_segments_async": (C.c_int, [vp, vp, u32, u64, u64p, C.POINTER(u32), u64p]),
    "nrg_log_exec": (C.c_int, [vp, u64, u64, vp, vp]),
    "nrg_log_exec_async": (C.c_int, [vp, u64, u64, vp, vp]),
    "nrg_log_state": (C.c_int, [vp, C.POINTER(LogInfo)]),
    "nrg_log_reset": (C.c_int, [vp]),
    "nrg_hashmap_get": (C.c_int, [vp, vp, u64, vp, vp]),
    "nrg_hashmap_get_async": (C.c_int, [vp, vp, u64, vp, vp]),
    "nrg_hashmap_round_async": (C.c_int, [vp, vp, u64, u32, vp, u64, vp, vp, vp, vp]),
    "nrg_stack_round_async": (C.c_int, [vp, vp, u64, u32, vp, vp]),
    "nrg_synth_round_async": (C.c_int, [vp, vp, u64, u32, vp, vp]),
    "nrg_hashmap_round_segments_async": (C.c_int, [vp, vp, u32, u64, u64p, C.POINTER(u32), u32, vp, u64, vp, vp,
                                                   vp, vp]),
    "nrg_hashmap_prefill": (C.c_int, [vp, vp, vp, u64]),
    "nrg_hashmap_prefill_range": (C.c_int, [vp, u64, u64]),
    "nrg_hashmap_size": (C.c_int, [vp, u64p]),
    "nrg_hashmap_dump": (C.c_int, [vp, vp, vp, u64, u64p]),
    "nrg_hashmap_digest": (C.c_int, [vp, vp]),
    "nrg_stack_init": (C.c_int, [vp, vp, u64]),
    "nrg_stack_peek": (C.c_int, [vp, C.POINTER(u32), C.POINTER(C.c_uint8)]),
    "nrg_stack_len": (C.c_int, [vp, u64p]),
    "nrg_stack_dump": (C.c_int, [vp, vp, u64, u64p]),
    "nrg_synth_read": (C.c_int, [vp, vp, u64, vp]),
    "nrg_synth_read_async": (C.c_int, [vp, vp, u64, vp]),
    "nrg_synth_dump": (C.c_int, [vp, vp, u64, u64p]),
    "nrg_dev_alloc": (C.c_int, [vp, u64, C.POINTER(vp)]),
    "nrg_dev_free": (C.c_int, [vp, vp]),
    "nrg_memcpy_h2d": (C.c_int, [vp, vp, vp, u64]),
    "nrg_memcpy_d2h": (C.c_int, [vp, vp, vp, u64]),
    "nrg_gen_uniform_async": (C.c_int, [vp, vp, u64, u64, u64]),
    "nrg_gen_raw_async": (C.c_int, [vp, vp, u64, u64]),
    "nrg_gen_puts_async": (C.c_int, [vp, vp, vp, vp, u64]),
    "nrg_gen_zipf_async": (C.c_int, [vp, vp, u64, u64, u64, C.c_double, C.c_int]),
    "nrg_gen_stack_ops_async": (C.c_int, [vp, vp, u64, u64]),
    "nrg_kernel_timing": (C.c_int, [vp, C.c_int]),
    "nrg_kernel_timing_only": (C.c_int, [vp, C.c_char_p]),
    "nrg_kernel_time": (C.c_int, [vp, C.c_char_p, u64p, C.POINTER(C.c_double)]),
    "nrg_group_unique_id": (C.c_int, [vp]),
    "nrg_group_join": (C.c_int, [vp, vp, C.c_int, C.c_int, C.POINTER(vp)]),
    "nrg_group_open": (C.c_int, [C.POINTER(C.c_int), C.c_int, C.POINTER(Config), C.POINTER(vp)]),
    "nrg_group_close": (C.c_int, [vp]),
    "nrg_group_info": (C.c_int, [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "nrg_group_replica": (vp, [vp, C.c_int]),
    "nrg_group_set_input_stream": (C.c_int, [vp, C.c_int, vp]),
    "nrg_group_round_async": (C.c_int, [vp, C.POINTER(Round), u64p]),
    "nrg_group_sync": (C.c_int, [vp]),
    "nrg_group_set_timeout": (C.c_int, [vp, u32]),
    "nrg_group_last_error": (C.c_char_p, [vp]),
    "nrg_combiner_open": (C.c_int, [vp, u32, C.POINTER(vp)]),
    "nrg_combiner_close": (C.c_int, [vp]),
    "nrg_combiner_register": (C.c_int, [vp, C.POINTER(u32)]),
    "nrg_combiner_put": (C.c_int, [vp, u32, vp, vp, u32, vp, vp]),
    "nrg_combiner_execute_mut": (C.c_int, [vp, u32, vp, u32, vp, vp]),
    "nrg_combiner_execute": (C.c_int, [vp, u32, vp, u32, vp, vp]),
    "nrg_combiner_get": (C.c_int, [vp, u32, vp, u32, vp, vp]),
    "nrg_combiner_stats": (C.c_int, [vp, u64p, u64p]),
    "nrg_key_owner": (C.c_uint32, [u64, C.c_uint32]),
    "nrg_hashmap_partition_async": (C.c_int, [vp, vp, u64, vp, u64, C.c_uint32, vp, vp, vp, vp, vp]),
    "nrg_route_back_async": (C.c_int, [vp, vp, vp, vp, u64, vp, vp]),
    "nrg_hashmap_prefill_partition": (C.c_int, [vp, u64, u64, C.c_uint32, C.c_uint32]),
    "nrg_group_partitioned_round": (C.c_int, [vp, C.POINTER(Round)]),
    "nrg_group_partitioned_round_async": (C.c_int, [vp, C.POINTER(Round)]),
    "nrg_group_partitioned_flush": (C.c_int, [vp]),
}

# include/nrgpu_testing.h (kernel unit-test hooks)
TEST_SIGNATURES = {
    "nrg_test_combiner_probe": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
    "nrg_test_combiner_times": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
    "nrg_test_sort_pairs": (C.c_int, [vp, vp, vp, u64, C.c_int, vp, vp]),
    "nrg_test_maxscan": (C.c_int, [vp, vp, vp, u64, vp]),
    "nrg_test_lds_add_order": (C.c_int, [vp, u32, u32, u32, vp]),
    "nrg_test_ring_read": (C.c_int, [vp, u64, vp]),
    "nrg_test_debug_read": (C.c_int, [vp, vp, u64]),
    "nrg_test_hm_skewed": (C.c_int, [vp, vp]),
    "nrg_test_set_knob": (C.c_int, [vp, C.c_int, u64]),
    "nrg_test_loopback_collectives": (C.c_int, [C.c_int]),
}

# nrg_test_set_knob knobs (include/nrgpu_testing.h): tuning and diagnostics of an open context
KNOBS = {"STAMP_MAX": 1, "SKEW_EVERY": 2, "EPOCH_LIMIT": 3, "K1": 4, "EXP": 6, "SY_SORT": 7,
         "PIPELINE": 8, "COMB_SPIN": 10, "COMB_DEPTH": 11,
         "SMALL_MAX": 12, "PART": 13, "STALL": 14, "COMB_GATHER": 15, "PA_TPB": 16, "COMB_SERVE": 17, "SY_FUSED": 18}

_lib = None


def load(path: str = LIB_PATH):
    """Load libnrgpu.so; raises OSError (loudly) if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(path):
            raise OSError(f"libnrgpu.so not built at {path}: run `make -C node-replication_amd` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
        L = C.CDLL(path)
        for name, (res, args) in {**SIGNATURES, **TEST_SIGNATURES}.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(code: int, what: str = ""):
    if code != NRG_OK:
        raise NrgError(code, what)
    return code


def default_config(kind: int) -> Config:
    cfg = Config()
    load().nrg_config_default(C.byref(cfg), kind)
    return cfg
