"""Native flat combining for many client threads (libnrgpu.so nrg_combiner_*).

Mirrors the reference's per-thread registration and synchronous execute / execute_mut
(nr/src/replica.rs:345-356, 404-433, 508-595; nr/src/context.rs:88-194): every call posts up to
32 ops of one thread into the open batch, and the combiner's own thread turns the batch into one
GPU round of the replica (writes, then reads) without waiting for the GPU. One call at a time per
token: a call on a token whose previous call is still waiting is refused (NRG_E_INVAL). Works for the three data structures (NrHashMap, Stack, AbstractDataStructure). ctypes
releases the GIL for the call, so Python threads combine for real.
"""
import ctypes as C

import numpy as np

from . import _lib as L
from .replica import PUT_DTYPE, STACK_OP_DTYPE, SYNTH_OP_DTYPE, SYNTH_RD_DTYPE

MAX_PENDING_OPS = 32  # nr/src/context.rs:12

# per kind: (write record dtype, write response dtype, read record dtype, read response dtype)
_KINDS = {
    L.NRG_DS_HASHMAP: (PUT_DTYPE, np.uint64, np.uint64, np.uint64),
    L.NRG_DS_STACK: (STACK_OP_DTYPE, np.uint32, None, np.uint32),
    L.NRG_DS_SYNTHETIC: (SYNTH_OP_DTYPE, np.uint64, SYNTH_RD_DTYPE, np.uint64),
}


class Combiner:
    """Flat combiner over one DeviceReplica (which it then drives exclusively)."""

    def __init__(self, replica, max_threads: int):
        self._lib = L.load()
        h = C.c_void_p()
        L.check(self._lib.nrg_combiner_open(replica.handle, max_threads, C.byref(h)), "nrg_combiner_open")
        self._h = h
        self.replica = replica
        self.kind = replica.kind

    def probe(self) -> dict:
        """(tests) the round server's words and the round counters (nrg_test_combiner_probe)."""
        out = (C.c_uint64 * 8)()
        L.check(self._lib.nrg_test_combiner_probe(self._h, out), "nrg_test_combiner_probe")
        keys = ("posted", "served", "exited", "session", "running", "completed", "launched", "open")
        return dict(zip(keys, (int(x) for x in out)))

    def register(self) -> int:
        """Replica::register: a thread token (NrgError NRG_E_CAPACITY past max_threads)."""
        t = C.c_uint32()
        L.check(self._lib.nrg_combiner_register(self._h, C.byref(t)), "nrg_combiner_register")
        return t.value

    def execute_mut(self, token: int, recs):
        """Replica::execute_mut for up to 32 log records of the replica's kind: (responses, Some flags)."""
        wdt, rdt, _, _ = _KINDS[self.kind]
        r = np.ascontiguousarray(recs, wdt)
        resp = np.zeros(len(r), rdt)
        some = np.zeros(len(r), np.uint8)
        L.check(self._lib.nrg_combiner_execute_mut(self._h, token, r.ctypes.data, len(r), resp.ctypes.data,
                                                   some.ctypes.data), "nrg_combiner_execute_mut")
        return resp, some

    def execute(self, token: int, reads=None, n: int = None):
        """Replica::execute for up to 32 reads (hashmap keys, synthetic nrg_synth_rd records, or
        n stack Peeks): (responses, Some flags)."""
        _, _, qdt, adt = _KINDS[self.kind]
        if qdt is None:
            q, cnt, ptr = None, int(n if n is not None else len(reads)), None
        else:
            q = np.ascontiguousarray(reads, qdt)
            cnt, ptr = len(q), q.ctypes.data
        resp = np.zeros(cnt, adt)
        some = np.zeros(cnt, np.uint8)
        L.check(self._lib.nrg_combiner_execute(self._h, token, ptr, cnt, resp.ctypes.data, some.ctypes.data),
                "nrg_combiner_execute")
        return resp, some

    def put(self, token: int, keys, vals):
        """execute_mut(Put(k, v)) for up to 32 ops: (previous values, Some flags)."""
        k = np.ascontiguousarray(keys, np.uint64)
        v = np.ascontiguousarray(vals, np.uint64)
        if len(v) != len(k):
            raise ValueError("keys and vals differ in length")
        if len(k) > MAX_PENDING_OPS:
            raise ValueError(f"at most {MAX_PENDING_OPS} ops per call (nr/src/context.rs:12)")
        prev = np.zeros(len(k), np.uint64)
        some = np.zeros(len(k), np.uint8)
        L.check(self._lib.nrg_combiner_put(self._h, token, k.ctypes.data, v.ctypes.data, len(k), prev.ctypes.data,
                                           some.ctypes.data), "nrg_combiner_put")
        return prev, some

    def get(self, token: int, keys):
        """execute(Get(k)) for up to 32 ops: (values, found flags)."""
        k = np.ascontiguousarray(keys, np.uint64)
        vals = np.zeros(len(k), np.uint64)
        found = np.zeros(len(k), np.uint8)
        L.check(self._lib.nrg_combiner_get(self._h, token, k.ctypes.data, len(k), vals.ctypes.data,
                                           found.ctypes.data), "nrg_combiner_get")
        return vals, found

    def stats(self):
        """(GPU rounds combined, ops they carried)."""
        r, o = C.c_uint64(), C.c_uint64()
        L.check(self._lib.nrg_combiner_stats(self._h, C.byref(r), C.byref(o)), "nrg_combiner_stats")
        return r.value, o.value

    def close(self):
        if getattr(self, "_h", None):
            self._lib.nrg_combiner_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
