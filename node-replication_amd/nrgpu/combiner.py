"""Native flat combining for many client threads (libnrgpu.so nrg_combiner_*).

Mirrors the reference's per-thread registration and synchronous execute / execute_mut
(nr/src/replica.rs:345-356, 414-433, 508-595; nr/src/context.rs:88-194): every call posts up to
32 ops of one thread, and whichever posting thread takes the combiner lock replays all posted
ops of all threads as one GPU round. ctypes releases the GIL for the call, so Python threads
combine for real.
"""
import ctypes as C

import numpy as np

from . import _lib as L

MAX_PENDING_OPS = 32  # nr/src/context.rs:12


class Combiner:
    """Flat combiner over one NrHashMap DeviceReplica (which it then drives exclusively)."""

    def __init__(self, replica, max_threads: int):
        self._lib = L.load()
        h = C.c_void_p()
        L.check(self._lib.nrg_combiner_open(replica.handle, max_threads, C.byref(h)), "nrg_combiner_open")
        self._h = h
        self.replica = replica

    def register(self) -> int:
        """Replica::register: a thread token (NrgError NRG_E_CAPACITY past max_threads)."""
        t = C.c_uint32()
        L.check(self._lib.nrg_combiner_register(self._h, C.byref(t)), "nrg_combiner_register")
        return t.value

    def put(self, token: int, keys, vals):
        """execute_mut(Put(k, v)) for up to 32 ops: (previous values, Some flags)."""
        k = np.ascontiguousarray(keys, np.uint64)
        v = np.ascontiguousarray(vals, np.uint64)
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
