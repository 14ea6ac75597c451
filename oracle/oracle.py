"""ctypes wrapper over the CPU oracle (oracle/build/libnroracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker / the timed CPU baseline; never by the product package.
The oracle restates the reference's sequential semantics (see nr_oracle.h for citations).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libnroracle.so")
_lib = None

u64p = C.POINTER(C.c_uint64)
u32p = C.POINTER(C.c_uint32)
u8p = C.POINTER(C.c_uint8)


def build() -> str:
    """Compile the oracle with its Makefile (gcc/g++ only)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        sig = {
            "orc_mix64": (C.c_uint64, [C.c_uint64]),
            "orc_sm64_at": (C.c_uint64, [C.c_uint64, C.c_uint64]),
            "orc_gen_raw": (None, [u64p, C.c_uint64, C.c_uint64]),
            "orc_gen_uniform": (None, [u64p, C.c_uint64, C.c_uint64, C.c_uint64]),
            "orc_gen_zipf": (None, [u64p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_double, C.c_int]),
            "orc_gen_hashmap_ops": (None, [u8p, u64p, u64p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32]),
            "orc_gen_stack_ops": (None, [u32p, u32p, C.c_uint64, C.c_uint64]),
            "orc_hm_new": (C.c_void_p, [C.c_uint64]),
            "orc_hm_free": (None, [C.c_void_p]),
            "orc_hm_insert": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64, u64p]),
            "orc_hm_get": (C.c_int, [C.c_void_p, C.c_uint64, u64p]),
            "orc_hm_len": (C.c_uint64, [C.c_void_p]),
            "orc_hm_prefill_range": (None, [C.c_void_p, C.c_uint64, C.c_uint64]),
            "orc_hm_replay": (None, [C.c_void_p, u64p, C.c_uint64, u64p, u8p]),
            "orc_hm_get_batch": (None, [C.c_void_p, u64p, C.c_uint64, u64p, u8p]),
            "orc_hm_run_mixed": (None, [C.c_void_p, u8p, u64p, u64p, C.c_uint64, u64p, u8p]),
            "orc_hm_dump_sorted": (C.c_uint64, [C.c_void_p, u64p, u64p]),
            "orc_hm_digest": (None, [C.c_void_p, u64p]),
            "orc_stack_new": (C.c_void_p, [u32p, C.c_uint64]),
            "orc_stack_free": (None, [C.c_void_p]),
            "orc_stack_replay": (None, [C.c_void_p, u32p, u32p, C.c_uint64, C.c_int, u32p, u8p]),
            "orc_stack_len": (C.c_uint64, [C.c_void_p]),
            "orc_stack_dump": (C.c_uint64, [C.c_void_p, u32p]),
            "orc_stack_peek": (C.c_int, [C.c_void_p, u32p]),
            "orc_synth_new": (C.c_void_p, [C.c_uint64] * 5),
            "orc_synth_free": (None, [C.c_void_p]),
            "orc_synth_replay": (None, [C.c_void_p, u64p, C.c_uint64, u64p]),
            "orc_synth_read": (None, [C.c_void_p, u64p, C.c_uint64, u64p]),
            "orc_synth_dump": (C.c_uint64, [C.c_void_p, u64p]),
            # control plane
            "orc_log_new": (C.c_void_p, [C.c_uint64]),
            "orc_log_default": (C.c_void_p, []),
            "orc_log_free": (None, [C.c_void_p]),
            "orc_log_entry_size": (C.c_uint64, []),
            "orc_log_const": (C.c_uint64, [C.c_int]),
            "orc_log_get": (C.c_uint64, [C.c_void_p, C.c_int]),
            "orc_log_set": (None, [C.c_void_p, C.c_int, C.c_uint64]),
            "orc_log_ltail": (C.c_uint64, [C.c_void_p, C.c_uint64]),
            "orc_log_set_ltail": (None, [C.c_void_p, C.c_uint64, C.c_uint64]),
            "orc_log_lmask": (C.c_int, [C.c_void_p, C.c_uint64]),
            "orc_log_index": (C.c_uint64, [C.c_void_p, C.c_uint64]),
            "orc_log_register": (C.c_long, [C.c_void_p]),
            "orc_log_entry": (C.c_int, [C.c_void_p, C.c_uint64, u64p, u64p]),
            "orc_log_append": (C.c_uint64, [C.c_void_p, u64p, C.c_uint64, C.c_uint64, u64p, u64p, C.c_uint64]),
            "orc_log_exec": (C.c_uint64, [C.c_void_p, C.c_uint64, u64p, u64p, C.c_uint64]),
            "orc_log_advance_head": (None, [C.c_void_p, C.c_uint64]),
            "orc_log_reset": (None, [C.c_void_p]),
            "orc_log_synced": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64]),
            "orc_log_get_ctail": (C.c_uint64, [C.c_void_p]),
            "orc_ctx_new": (C.c_void_p, []),
            "orc_ctx_free": (None, [C.c_void_p]),
            "orc_ctx_enqueue": (C.c_int, [C.c_void_p, C.c_uint64]),
            "orc_ctx_enqueue_resps": (None, [C.c_void_p, u64p, C.c_uint64]),
            "orc_ctx_ops": (C.c_uint64, [C.c_void_p, u64p, C.c_uint64]),
            "orc_ctx_res": (C.c_int, [C.c_void_p, u64p]),
            "orc_ctx_get": (C.c_uint64, [C.c_void_p, C.c_int]),
            "orc_ctx_set": (None, [C.c_void_p, C.c_int, C.c_uint64]),
            "orc_rep_new": (C.c_void_p, [C.c_uint64]),
            "orc_rep_free": (None, [C.c_void_p]),
            "orc_rep_register": (C.c_long, [C.c_void_p]),
            "orc_rep_get": (C.c_uint64, [C.c_void_p, C.c_int]),
            "orc_rep_set": (None, [C.c_void_p, C.c_int, C.c_uint64]),
            "orc_rep_make_pending": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint64]),
            "orc_rep_try_combine": (None, [C.c_void_p, C.c_uint64]),
            "orc_rep_execute_mut": (C.c_uint64, [C.c_void_p, C.c_uint64, C.c_uint64]),
            "orc_rep_execute": (C.c_uint64, [C.c_void_p, C.c_uint64, C.c_uint64]),
            "orc_rep_get_response": (C.c_uint64, [C.c_void_p, C.c_uint64]),
            "orc_rep_ctx_res": (C.c_int, [C.c_void_p, C.c_uint64, u64p]),
            "orc_rep_log_append_exec": (None, [C.c_void_p, u64p, C.c_uint64, C.c_uint64]),
            "orc_nr_hashmap_bench": (C.c_int, [C.c_uint32, C.POINTER(C.c_int), u32p, C.c_uint32, C.c_double,
                                                C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64,
                                                C.c_uint64, C.c_void_p]),
            "orc_nr_stack_bench": (C.c_int, [C.c_uint32, C.POINTER(C.c_int), u32p, C.c_uint32, C.c_double,
                                              C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p]),
            "orc_nr_synth_bench": (C.c_int, [C.c_uint32, C.POINTER(C.c_int), u32p, C.c_uint32, C.c_double,
                                              C.c_uint64, C.c_uint64, C.c_uint64, C.c_void_p]),
            "orc_nr_stack_run": (C.c_uint64, [u32p, C.c_uint64, u32p, u32p, C.c_uint64, u64p, u32p, C.c_uint64]),
            "orc_nr_synth_run": (None, [u64p, C.c_uint64, u64p, C.c_uint64, u64p, u64p, u64p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(t)


# ---- generators ---------------------------------------------------------------------
def mix64(x: int) -> int:
    return int(lib().orc_mix64(x))


def gen_raw(n: int, seed: int) -> np.ndarray:
    out = np.empty(n, np.uint64)
    lib().orc_gen_raw(_p(out, u64p), n, seed)
    return out


def gen_uniform(n: int, seed: int, span: int) -> np.ndarray:
    out = np.empty(n, np.uint64)
    lib().orc_gen_uniform(_p(out, u64p), n, seed, span)
    return out


def gen_zipf(n: int, seed: int, N: int, theta: float = 0.99, scramble: bool = False) -> np.ndarray:
    out = np.empty(n, np.uint64)
    lib().orc_gen_zipf(_p(out, u64p), n, seed, N, theta, int(scramble))
    return out


def gen_hashmap_ops(n: int, seed: int, span: int, write_ratio: int):
    is_put = np.empty(n, np.uint8)
    keys = np.empty(n, np.uint64)
    vals = np.empty(n, np.uint64)
    lib().orc_gen_hashmap_ops(_p(is_put, u8p), _p(keys, u64p), _p(vals, u64p), n, seed, span, write_ratio)
    return is_put, keys, vals


def gen_stack_ops(n: int, seed: int):
    vals = np.empty(n, np.uint32)
    ops = np.empty(n, np.uint32)
    lib().orc_gen_stack_ops(_p(vals, u32p), _p(ops, u32p), n, seed)
    return vals, ops


# ---- NrHashMap ------------------------------------------------------------------------
class HashMap:
    """Sequential std::HashMap<u64,u64> restatement (benches/hashmap.rs:77-122)."""

    def __init__(self, initial_capacity: int = 16):
        self._m = lib().orc_hm_new(initial_capacity)

    def __del__(self):
        if getattr(self, "_m", None):
            lib().orc_hm_free(self._m)
            self._m = None

    def __len__(self):
        return int(lib().orc_hm_len(self._m))

    def insert(self, k: int, v: int):
        pv = C.c_uint64(0)
        f = lib().orc_hm_insert(self._m, k, v, C.byref(pv))
        return int(pv.value) if f else None

    def get(self, k: int):
        v = C.c_uint64(0)
        f = lib().orc_hm_get(self._m, k, C.byref(v))
        return int(v.value) if f else None

    def prefill_range(self, n: int, off: int = 1):
        lib().orc_hm_prefill_range(self._m, n, off)

    def replay(self, keys: np.ndarray, vals: np.ndarray, want_prev: bool = True):
        W = len(keys)
        kv = np.empty(2 * W, np.uint64)
        kv[0::2] = keys
        kv[1::2] = vals
        prev = np.zeros(W, np.uint64)
        found = np.zeros(W, np.uint8)
        lib().orc_hm_replay(self._m, _p(kv, u64p), W, _p(prev, u64p), _p(found, u8p))
        return prev, found

    def get_batch(self, keys: np.ndarray):
        keys = np.ascontiguousarray(keys, np.uint64)
        vals = np.zeros(len(keys), np.uint64)
        found = np.zeros(len(keys), np.uint8)
        lib().orc_hm_get_batch(self._m, _p(keys, u64p), len(keys), _p(vals, u64p), _p(found, u8p))
        return vals, found

    def run_mixed(self, is_put, keys, vals):
        n = len(keys)
        resp = np.zeros(n, np.uint64)
        some = np.zeros(n, np.uint8)
        lib().orc_hm_run_mixed(self._m, _p(is_put, u8p), _p(keys, u64p), _p(vals, u64p), n,
                               _p(resp, u64p), _p(some, u8p))
        return resp, some

    def dump_sorted(self):
        n = len(self)
        k = np.empty(max(n, 1), np.uint64)
        v = np.empty(max(n, 1), np.uint64)
        m = lib().orc_hm_dump_sorted(self._m, _p(k, u64p), _p(v, u64p))
        return k[:m], v[:m]

    def digest(self):
        out = np.zeros(3, np.uint64)
        lib().orc_hm_digest(self._m, _p(out, u64p))
        return tuple(int(x) for x in out)


# ---- Stack ----------------------------------------------------------------------------
class Stack:
    def __init__(self, init=None):
        init = np.ascontiguousarray(np.asarray(init if init is not None else [], np.uint32))
        self._s = lib().orc_stack_new(_p(init, u32p), len(init))

    def __del__(self):
        if getattr(self, "_s", None):
            lib().orc_stack_free(self._s)
            self._s = None

    def replay(self, vals, ops, push_resp: bool = False):
        vals = np.ascontiguousarray(vals, np.uint32)
        ops = np.ascontiguousarray(ops, np.uint32)
        n = len(ops)
        resp = np.zeros(n, np.uint32)
        some = np.zeros(n, np.uint8)
        lib().orc_stack_replay(self._s, _p(vals, u32p), _p(ops, u32p), n, int(push_resp), _p(resp, u32p),
                               _p(some, u8p))
        return resp, some

    def __len__(self):
        return int(lib().orc_stack_len(self._s))

    def dump(self):
        out = np.empty(max(len(self), 1), np.uint32)
        n = lib().orc_stack_dump(self._s, _p(out, u32p))
        return out[:n]

    def peek(self):
        v = C.c_uint32(0)
        return int(v.value) if lib().orc_stack_peek(self._s, C.byref(v)) else None


# ---- AbstractDataStructure ---------------------------------------------------------------
class Synthetic:
    def __init__(self, n=200_000, cold_reads=20, cold_writes=5, hot_reads=2, hot_writes=1):
        self.n = n
        self._s = lib().orc_synth_new(n, cold_reads, cold_writes, hot_reads, hot_writes)

    def __del__(self):
        if getattr(self, "_s", None):
            lib().orc_synth_free(self._s)
            self._s = None

    def replay(self, ops: np.ndarray):
        """ops: (n, 4) uint64 rows {tid, r1, r2, op}"""
        ops = np.ascontiguousarray(ops, np.uint64)
        n = ops.shape[0]
        resp = np.zeros(n, np.uint64)
        lib().orc_synth_replay(self._s, _p(ops, u64p), n, _p(resp, u64p))
        return resp

    def read(self, ops: np.ndarray):
        ops = np.ascontiguousarray(ops, np.uint64)
        n = ops.shape[0]
        out = np.zeros(n, np.uint64)
        lib().orc_synth_read(self._s, _p(ops, u64p), n, _p(out, u64p))
        return out

    def dump(self):
        out = np.empty(self.n, np.uint64)
        lib().orc_synth_dump(self._s, _p(out, u64p))
        return out


class BenchResult(C.Structure):
    _fields_ = [("seconds", C.c_double), ("ops", C.c_uint64), ("writes", C.c_uint64), ("reads", C.c_uint64)]


def nr_hashmap_bench(cpus, cpu_replica, duration_s, write_ratio, key_space, prefill, nop, seed,
                     log_bytes=32 << 20):
    """Multi-threaded C++ restatement of the nr scale-out bench (benches/hashmap.rs:226-259)."""
    n = len(cpus)
    ca = (C.c_int * n)(*cpus)
    ra = (C.c_uint32 * n)(*cpu_replica)
    res = BenchResult()
    nrep = max(cpu_replica) + 1
    rc = lib().orc_nr_hashmap_bench(nrep, ca, ra, n, duration_s, write_ratio, key_space, prefill, nop, seed,
                                    log_bytes, C.byref(res))
    if rc != 0:
        raise RuntimeError("orc_nr_hashmap_bench failed")
    return res


def _scale_out(fn, cpus, cpu_replica, duration_s, *args):
    n = len(cpus)
    ca = (C.c_int * n)(*cpus)
    ra = (C.c_uint32 * n)(*cpu_replica)
    res = BenchResult()
    rc = getattr(lib(), fn)(max(cpu_replica) + 1, ca, ra, n, duration_s, *args, C.byref(res))
    if rc != 0:
        raise RuntimeError(fn + " failed")
    return res


def nr_stack_bench(cpus, cpu_replica, duration_s, nop, seed, log_bytes=32 << 20):
    """Stack scale-out through the C++ restatement of nr (benches/stack.rs:115-134)."""
    return _scale_out("orc_nr_stack_bench", cpus, cpu_replica, duration_s, nop, seed, log_bytes)


def nr_synth_bench(cpus, cpu_replica, duration_s, nop, seed, log_bytes=32 << 20):
    """Synthetic scale-out through the C++ restatement of nr (benches/synthetic.rs:296-335)."""
    return _scale_out("orc_nr_synth_bench", cpus, cpu_replica, duration_s, nop, seed, log_bytes)


def nr_stack_run(init, vals, kinds):
    """One thread's execute_mut stream through Replica<Stack> of the nr restatement: returns
    (responses as Option<u32> with bit 32 = Some, final storage)."""
    init = np.ascontiguousarray(init, np.uint32)
    vals = np.ascontiguousarray(vals, np.uint32)
    kinds = np.ascontiguousarray(kinds, np.uint32)
    n = vals.shape[0]
    resp = np.zeros(n, np.uint64)
    cap = init.shape[0] + n
    fin = np.zeros(max(cap, 1), np.uint32)
    ln = lib().orc_nr_stack_run(_p(init, u32p), init.shape[0], _p(vals, u32p), _p(kinds, u32p), n,
                                _p(resp, u64p), _p(fin, u32p), cap)
    return resp, fin[:ln]


def nr_synth_run(ops4, reads3):
    """One thread's execute_mut stream then execute reads through Replica<AbstractDataStructure>
    of the nr restatement: (write responses, read responses, final storage)."""
    ops4 = np.ascontiguousarray(ops4, np.uint64)
    reads3 = np.ascontiguousarray(reads3, np.uint64).reshape(-1, 3)
    resp = np.zeros(ops4.shape[0], np.uint64)
    rresp = np.zeros(max(reads3.shape[0], 1), np.uint64)
    fin = np.zeros(200_000, np.uint64)
    lib().orc_nr_synth_run(_p(ops4, u64p), ops4.shape[0], _p(reads3, u64p), reads3.shape[0], _p(resp, u64p),
                           _p(rresp, u64p), _p(fin, u64p))
    return resp, rresp[:reads3.shape[0]], fin
