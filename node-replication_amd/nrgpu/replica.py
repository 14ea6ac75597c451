"""Host side of the MI355X NR replica, mirroring the `nr` crate's API over the C ABI.

  DeviceReplica   one nrg_ctx: a replica on one GPU (data structure + HBM log ring)
  Log             nr::Log         (nr/src/log.rs)       — the logical shared log; each GPU
                                   replica holds a physical copy in HBM
  Replica         nr::Replica<D>  (nr/src/replica.rs)   — register / execute_mut / execute /
                                   sync / verify, with flat combining of the registered
                                   threads' pending ops into one log append + one replay
  ReplicaToken    nr::ReplicaToken
  NrHashMap, Stack, AbstractDataStructure — the Dispatch plug-ins of the reference
                                   (benches/hashmap.rs, benches/stack.rs, benches/synthetic.rs)
"""
from __future__ import annotations

import ctypes as C
import sys
import threading
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import _lib as L

PUT_DTYPE = np.dtype([("key", "<u8"), ("val", "<u8")])
STACK_OP_DTYPE = np.dtype([("val", "<u4"), ("op", "<u4")])
SYNTH_OP_DTYPE = np.dtype([("tid", "<u8"), ("r1", "<u8"), ("r2", "<u8"), ("op", "<u8")])
SYNTH_RD_DTYPE = np.dtype([("tid", "<u8"), ("r1", "<u8"), ("r2", "<u8")])

# nr/src/log.rs:22,26,36 ; nr/src/context.rs:12 ; nr/src/replica.rs:56
DEFAULT_LOG_BYTES = 32 * 1024 * 1024
MAX_REPLICAS = 192
MAX_PENDING_OPS = 32
MAX_THREADS_PER_REPLICA = 256
GC_FROM_HEAD = MAX_PENDING_OPS * MAX_THREADS_PER_REPLICA


def _ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data)


def _dptr(t) -> C.c_void_p:
    """device pointer of a torch tensor / int / None"""
    if t is None:
        return C.c_void_p(0)
    if isinstance(t, int):
        return C.c_void_p(t)
    return C.c_void_p(t.data_ptr())


def _stream_ordered(fn):
    """Stream-ordering contract of every `*_device` helper (and join): the call is ordered AFTER
    all work already queued on torch's current stream (so buffers torch filled or copied there
    are ready), and torch's current stream is ordered AFTER the work the call queued on this
    replica's stream (so torch reads of the outputs see them). When the replica already runs on
    torch's current stream (use_torch_stream) this is free; otherwise two events cross the
    streams. With config.pipeline = 1 a round's deferred outputs are complete only after join(),
    which is ordered the same way. Without this, a replica on its own non-blocking stream
    (nrg_open's default, include/nrgpu.h nrg_set_stream) races torch's null-stream fills."""

    def wrapped(self, *a, **kw):
        cross = self._cross_streams()
        if cross is None:
            return fn(self, *a, **kw)
        cur, mine = cross
        mine.wait_stream(cur)
        try:
            return fn(self, *a, **kw)
        finally:
            cur.wait_stream(mine)

    wrapped.__name__ = fn.__name__
    wrapped.__doc__ = fn.__doc__
    return wrapped


class DeviceReplica:
    """Thin owner of one nrg_ctx (one replica in one GPU's HBM).

    Stream contract: the replica queues its GPU work on its own stream (nrg_own_stream, not
    ordered with the null stream) until use_torch_stream / set_stream says otherwise. Every
    `*_device` method and join() is nevertheless ordered with torch's current stream in both
    directions (`_stream_ordered`), so torch tensors may be filled, passed and read back on
    torch's stream without extra synchronisation. Host-pointer methods are synchronous."""

    def __init__(self, kind: int, device: int = 0, knobs: Optional[dict] = None, **cfg):
        """`cfg`: nrg_config fields; `knobs`: {name: value} of nrg_test_set_knob (tuning and
        diagnostics, include/nrgpu_testing.h), applied right after nrg_open."""
        lib = L.load()
        self.kind = kind
        self.device = device
        c = L.default_config(kind)
        for k, v in cfg.items():
            if not hasattr(c, k):
                raise TypeError(f"unknown config field {k}")
            setattr(c, k, v)
        self.cfg = c
        h = C.c_void_p()
        L.check(lib.nrg_open(device, C.byref(c), C.byref(h)), "nrg_open")
        self._h = h
        self._lib = lib
        for k, v in (knobs or {}).items():
            self.set_knob(k, v)

    def set_knob(self, name: str, value: int):
        """nrg_test_set_knob: a tuning/diagnostic knob by name (L.KNOBS) on this open context."""
        L.check(self._lib.nrg_test_set_knob(self._h, L.KNOBS[name], int(value)), f"knob {name}")

    # -- lifetime ------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None):
            self._lib.nrg_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream_ptr: int):
        L.check(self._lib.nrg_set_stream(self._h, C.c_void_p(stream_ptr)), "nrg_set_stream")

    def use_torch_stream(self):
        """Order this replica's work with torch's current stream on its device (the null
        stream when torch is on its default stream)."""
        import torch

        self.set_stream(torch.cuda.current_stream(self.device).cuda_stream)

    def use_own_stream(self):
        self.set_stream(self._lib.nrg_own_stream(self._h) or 0)

    def _cross_streams(self):
        """(torch's current stream, this replica's stream as a torch stream) when the two differ
        and torch drives a GPU; None when no ordering is needed."""
        torch = sys.modules.get("torch")
        if torch is None or not torch.cuda.is_available():
            return None
        cur = torch.cuda.current_stream(self.device)
        mine = self._lib.nrg_get_stream(self._h) or 0
        if cur.cuda_stream == mine:
            return None
        cache = getattr(self, "_ext_stream", None)
        if cache is None or cache[0] != mine:
            s = (torch.cuda.default_stream(self.device) if mine == 0
                 else torch.cuda.ExternalStream(mine, device=torch.device("cuda", self.device)))
            cache = self._ext_stream = (mine, s)
        return cur, cache[1]

    def sync(self):
        L.check(self._lib.nrg_sync(self._h), "nrg_sync")

    @_stream_ordered
    def join(self):
        """Order outstanding side-stream reads (pipeline=1) on this replica's stream.
        Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        L.check(self._lib.nrg_join(self._h), "nrg_join")

    # -- log -----------------------------------------------------------------------
    def log_state(self) -> dict:
        info = L.LogInfo()
        L.check(self._lib.nrg_log_state(self._h, C.byref(info)))
        return {f: getattr(info, f) for f, _ in L.LogInfo._fields_}

    def log_append(self, recs: np.ndarray, origin: int) -> int:
        recs = np.ascontiguousarray(recs)
        first = C.c_uint64()
        L.check(self._lib.nrg_log_append(self._h, _ptr(recs), len(recs), origin, C.byref(first)), "append")
        return first.value

    @_stream_ordered
    def log_append_device(self, d_recs, n: int, origin: int) -> int:
        """Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        first = C.c_uint64()
        L.check(self._lib.nrg_log_append_async(self._h, _dptr(d_recs), n, origin, C.byref(first)), "append")
        return first.value

    @_stream_ordered
    def log_append_segments(self, d_base, seg_stride: int, lens: Sequence[int], origins: Sequence[int]):
        """Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        key = (tuple(lens), tuple(origins))
        if getattr(self, "_seg_key", None) != key:  # marshalled once per distinct round shape
            nseg = len(lens)
            self._seg_key = key
            self._seg_arrays = ((C.c_uint64 * nseg)(*lens), (C.c_uint32 * nseg)(*origins), nseg)
        la, oa, nseg = self._seg_arrays
        fa = (C.c_uint64 * nseg)()
        L.check(self._lib.nrg_log_append_segments_async(self._h, _dptr(d_base), nseg, seg_stride, la, oa, fa),
                "append_segments")
        return list(fa)

    def _resp_dtype(self):
        return np.uint32 if self.kind == L.NRG_DS_STACK else np.uint64

    def log_exec(self, resp_lo: int = 0, resp_hi: int = 0):
        n = resp_hi - resp_lo
        resp = np.zeros(max(n, 1), self._resp_dtype())
        some = np.zeros(max(n, 1), np.uint8)
        if n > 0:
            L.check(self._lib.nrg_log_exec(self._h, resp_lo, resp_hi, _ptr(resp), _ptr(some)), "exec")
        else:
            L.check(self._lib.nrg_log_exec(self._h, 0, 0, None, None), "exec")
        return resp[:n], some[:n]

    @_stream_ordered
    def log_exec_device(self, resp_lo=0, resp_hi=0, d_resp=None, d_some=None):
        """Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        L.check(self._lib.nrg_log_exec_async(self._h, resp_lo, resp_hi, _dptr(d_resp), _dptr(d_some)), "exec")

    @_stream_ordered
    def st_round_device(self, d_ops, n: int, origin: int, d_resp=None, d_some=None):
        """Replica::combine for one stack batch on device buffers: append + exec in one replay
        pass (nrg_stack_round_async); Pop responses for these ops into d_resp / d_some.
        Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        L.check(self._lib.nrg_stack_round_async(self._h, _dptr(d_ops), n, origin, _dptr(d_resp), _dptr(d_some)),
                "stack_round")

    @_stream_ordered
    def sy_round_device(self, d_ops, n: int, origin: int, d_resp=None, d_some=None):
        """Replica::combine for one synthetic batch on device buffers (nrg_synth_round_async).
        Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        L.check(self._lib.nrg_synth_round_async(self._h, _dptr(d_ops), n, origin, _dptr(d_resp), _dptr(d_some)),
                "synth_round")

    def log_reset(self):
        L.check(self._lib.nrg_log_reset(self._h))

    # -- hashmap -------------------------------------------------------------------
    def hm_get(self, keys: np.ndarray):
        keys = np.ascontiguousarray(keys, np.uint64)
        n = len(keys)
        vals = np.zeros(max(n, 1), np.uint64)
        found = np.zeros(max(n, 1), np.uint8)
        L.check(self._lib.nrg_hashmap_get(self._h, _ptr(keys), n, _ptr(vals), _ptr(found)), "get")
        return vals[:n], found[:n]

    @_stream_ordered
    def hm_get_device(self, d_keys, n, d_vals, d_found):
        """Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        L.check(self._lib.nrg_hashmap_get_async(self._h, _dptr(d_keys), n, _dptr(d_vals), _dptr(d_found)), "get")

    @_stream_ordered
    def hm_round_device(self, d_puts, W, origin, d_get_keys, R, d_get_vals, d_get_found, d_prev=None,
                        d_prev_found=None):
        """Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        L.check(self._lib.nrg_hashmap_round_async(self._h, _dptr(d_puts), W, origin, _dptr(d_get_keys), R,
                                                  _dptr(d_get_vals), _dptr(d_get_found), _dptr(d_prev),
                                                  _dptr(d_prev_found)), "round")

    @_stream_ordered
    def hm_round_segments_device(self, d_base, seg_stride, lens, origins, resp_seg, d_get_keys, R, d_get_vals,
                                 d_get_found, d_prev=None, d_prev_found=None):
        """Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        key = (tuple(lens), tuple(origins))
        if getattr(self, "_seg_key", None) != key:  # marshalled once per distinct round shape
            nseg = len(lens)
            self._seg_key = key
            self._seg_arrays = ((C.c_uint64 * nseg)(*lens), (C.c_uint32 * nseg)(*origins), nseg)
        la, oa, nseg = self._seg_arrays
        L.check(self._lib.nrg_hashmap_round_segments_async(
            self._h, _dptr(d_base), nseg, seg_stride, la, oa, resp_seg, _dptr(d_get_keys), R, _dptr(d_get_vals),
            _dptr(d_get_found), _dptr(d_prev), _dptr(d_prev_found)), "round_segments")

    def hm_prefill(self, keys: np.ndarray, vals: np.ndarray):
        keys = np.ascontiguousarray(keys, np.uint64)
        vals = np.ascontiguousarray(vals, np.uint64)
        L.check(self._lib.nrg_hashmap_prefill(self._h, _ptr(keys), _ptr(vals), len(keys)), "prefill")

    def hm_prefill_range(self, n: int, off: int = 1):
        L.check(self._lib.nrg_hashmap_prefill_range(self._h, n, off), "prefill_range")

    def hm_prefill_partition(self, n: int, off: int, part: int, parts: int):
        """NrHashMap::default restricted to key partition `part` of `parts` (nrg_key_owner)."""
        L.check(self._lib.nrg_hashmap_prefill_partition(self._h, n, off, part, parts), "prefill_partition")

    @_stream_ordered
    def hm_partition_device(self, d_puts, W, d_keys, R, parts, d_puts_out, d_put_pos, d_keys_out, d_get_pos, d_counts):
        """Stable partition of a round's Puts and Get keys by owner (nrg_hashmap_partition_async).
        Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        L.check(self._lib.nrg_hashmap_partition_async(self._h, _dptr(d_puts), W, _dptr(d_keys), R, parts,
                                                      _dptr(d_puts_out), _dptr(d_put_pos), _dptr(d_keys_out),
                                                      _dptr(d_get_pos), _dptr(d_counts)), "partition")

    @_stream_ordered
    def route_back_device(self, d_src, d_src8, d_pos, n, d_dst, d_dst8):
        """Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        L.check(self._lib.nrg_route_back_async(self._h, _dptr(d_src), _dptr(d_src8), _dptr(d_pos), n, _dptr(d_dst),
                                               _dptr(d_dst8)), "route_back")

    def partitioned_replay(self, puts, keys, want_prev: bool):
        """One owner's share of a key-partitioned round (nrgpu.parallel.PartitionedHashMap): replay
        the received Puts [p, 2] in the given (rank) order, answer the received Gets after them."""
        import torch

        dev = torch.device("cuda", self.device) if torch.cuda.is_available() else torch.device("cpu")
        p = puts.reshape(-1, 2).to(dev).contiguous()
        k = keys.reshape(-1).to(dev).contiguous()
        n, r = p.shape[0], k.shape[0]
        vals = torch.zeros(r, dtype=torch.int64, device=dev)
        found = torch.zeros(r, dtype=torch.uint8, device=dev)
        pv = torch.zeros(n, dtype=torch.int64, device=dev) if want_prev else None
        pf = torch.zeros(n, dtype=torch.uint8, device=dev) if want_prev else None
        self.use_torch_stream()
        self.hm_round_device(p, n, int(self.cfg.replica_id) or 1, k, r, vals, found, pv, pf)
        self.join()
        torch.cuda.synchronize(dev)
        return vals, found, pv, pf

    def hm_size(self) -> int:
        n = C.c_uint64()
        L.check(self._lib.nrg_hashmap_size(self._h, C.byref(n)))
        return n.value

    def hm_dump(self):
        """(keys, vals) sorted by key"""
        n = self.hm_size()
        k = np.zeros(max(n, 1), np.uint64)
        v = np.zeros(max(n, 1), np.uint64)
        m = C.c_uint64()
        L.check(self._lib.nrg_hashmap_dump(self._h, _ptr(k), _ptr(v), n, C.byref(m)), "dump")
        k, v = k[: m.value], v[: m.value]
        o = np.argsort(k, kind="stable")
        return k[o], v[o]

    def hm_digest(self):
        out = np.zeros(3, np.uint64)
        L.check(self._lib.nrg_hashmap_digest(self._h, _ptr(out)), "digest")
        return tuple(int(x) for x in out)

    # -- stack ---------------------------------------------------------------------
    def st_init(self, vals):
        vals = np.ascontiguousarray(np.asarray(vals, np.uint32))
        L.check(self._lib.nrg_stack_init(self._h, _ptr(vals), len(vals)), "stack_init")

    def st_peek(self):
        v = C.c_uint32()
        s = C.c_uint8()
        L.check(self._lib.nrg_stack_peek(self._h, C.byref(v), C.byref(s)), "peek")
        return int(v.value) if s.value else None

    def st_len(self) -> int:
        n = C.c_uint64()
        L.check(self._lib.nrg_stack_len(self._h, C.byref(n)))
        return n.value

    def st_dump(self) -> np.ndarray:
        n = self.st_len()
        out = np.zeros(max(n, 1), np.uint32)
        m = C.c_uint64()
        L.check(self._lib.nrg_stack_dump(self._h, _ptr(out), n, C.byref(m)), "stack_dump")
        return out[: m.value]

    # -- synthetic -----------------------------------------------------------------
    def sy_read(self, ops: np.ndarray) -> np.ndarray:
        ops = np.ascontiguousarray(ops, SYNTH_RD_DTYPE)
        out = np.zeros(max(len(ops), 1), np.uint64)
        L.check(self._lib.nrg_synth_read(self._h, _ptr(ops), len(ops), _ptr(out)), "synth_read")
        return out[: len(ops)]

    def sy_dump(self) -> np.ndarray:
        n = self.cfg.synth_n
        out = np.zeros(n, np.uint64)
        m = C.c_uint64()
        L.check(self._lib.nrg_synth_dump(self._h, _ptr(out), n, C.byref(m)), "synth_dump")
        return out

    # -- generators / timing -------------------------------------------------------
    @_stream_ordered
    def gen_uniform_device(self, d_out, n, seed, span):
        """Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        L.check(self._lib.nrg_gen_uniform_async(self._h, _dptr(d_out), n, seed, span))

    @_stream_ordered
    def gen_raw_device(self, d_out, n, seed):
        """Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        L.check(self._lib.nrg_gen_raw_async(self._h, _dptr(d_out), n, seed))

    @_stream_ordered
    def gen_zipf_device(self, d_out, n, seed, N, theta=0.99, scramble=False):
        """Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        L.check(self._lib.nrg_gen_zipf_async(self._h, _dptr(d_out), n, seed, N, float(theta), int(scramble)), "zipf")

    @_stream_ordered
    def gen_stack_ops_device(self, d_out, n, seed):
        """Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        L.check(self._lib.nrg_gen_stack_ops_async(self._h, _dptr(d_out), n, seed), "stack ops")

    @_stream_ordered
    def gen_puts_device(self, d_out, d_keys, d_vals, n):
        """Ordered after torch's current stream, and torch's stream after it (_stream_ordered)."""
        L.check(self._lib.nrg_gen_puts_async(self._h, _dptr(d_out), _dptr(d_keys), _dptr(d_vals), n))

    def kernel_timing(self, enable: bool = True, only: Optional[str] = None, every: int = 1):
        """HIP-event timing of kernel `only` (all if None), on every `every`-th launch."""
        L.check(self._lib.nrg_kernel_timing_only(self._h, (only or "").encode()))
        L.check(self._lib.nrg_kernel_timing(self._h, max(1, int(every)) if enable else 0))

    def kernel_time(self, name: str):
        n = C.c_uint64()
        ms = C.c_double()
        L.check(self._lib.nrg_kernel_time(self._h, name.encode(), C.byref(n), C.byref(ms)))
        return n.value, ms.value


# =====================================================================================
# Dispatch plug-ins (the reference's data structures) and their operations
# =====================================================================================
@dataclass(frozen=True)
class Put:  # benches/hashmap.rs:52-56
    key: int
    val: int


@dataclass(frozen=True)
class Get:  # benches/hashmap.rs:59-63
    key: int


@dataclass(frozen=True)
class Push:  # benches/stack.rs:22-28
    val: int


@dataclass(frozen=True)
class Pop:
    pass


@dataclass(frozen=True)
class Peek:  # nr/tests/stack.rs:26-29
    pass


@dataclass(frozen=True)
class WriteOnly:  # benches/synthetic.rs:33-39
    tid: int
    r1: int
    r2: int


@dataclass(frozen=True)
class ReadWrite:
    tid: int
    r1: int
    r2: int


@dataclass(frozen=True)
class ReadOnly:  # benches/synthetic.rs:28-31
    tid: int
    r1: int
    r2: int


class NrHashMap:
    """NrHashMap: HashMap<u64,u64>; Put -> previous value (nr/examples/hashmap.rs:46-50)."""

    kind = L.NRG_DS_HASHMAP
    rec_dtype = PUT_DTYPE

    @staticmethod
    def encode(ops: Sequence[Put]) -> np.ndarray:
        r = np.zeros(len(ops), PUT_DTYPE)
        r["key"] = [o.key for o in ops]
        r["val"] = [o.val for o in ops]
        return r

    @staticmethod
    def decode(resp, some) -> list:
        return [int(v) if s else None for v, s in zip(resp, some)]

    @staticmethod
    def read_batch(dev: DeviceReplica, ops: Sequence[Get]) -> list:
        v, f = dev.hm_get(np.array([o.key for o in ops], np.uint64))
        return [int(a) if b else None for a, b in zip(v, f)]

    @staticmethod
    def snapshot(dev: DeviceReplica):
        k, v = dev.hm_dump()
        return dict(zip(k.tolist(), v.tolist()))


class Stack:
    """Stack: Vec<u32>; Push -> None (or Some(v) with push_resp=1), Pop -> Option<u32>."""

    kind = L.NRG_DS_STACK
    rec_dtype = STACK_OP_DTYPE

    @staticmethod
    def encode(ops) -> np.ndarray:
        r = np.zeros(len(ops), STACK_OP_DTYPE)
        r["val"] = [o.val if isinstance(o, Push) else 0 for o in ops]
        r["op"] = [L.NRG_STACK_PUSH if isinstance(o, Push) else L.NRG_STACK_POP for o in ops]
        return r

    @staticmethod
    def decode(resp, some) -> list:
        return [int(v) if s else None for v, s in zip(resp, some)]

    @staticmethod
    def read_batch(dev: DeviceReplica, ops) -> list:
        top = dev.st_peek()
        return [top for _ in ops]

    @staticmethod
    def snapshot(dev: DeviceReplica):
        return dev.st_dump().tolist()


class AbstractDataStructure:
    """benches/synthetic.rs AbstractDataStructure::new(n, 20, 5, 2, 1)."""

    kind = L.NRG_DS_SYNTHETIC
    rec_dtype = SYNTH_OP_DTYPE

    @staticmethod
    def encode(ops) -> np.ndarray:
        r = np.zeros(len(ops), SYNTH_OP_DTYPE)
        r["tid"] = [o.tid for o in ops]
        r["r1"] = [o.r1 for o in ops]
        r["r2"] = [o.r2 for o in ops]
        r["op"] = [L.NRG_SYNTH_READ_WRITE if isinstance(o, ReadWrite) else L.NRG_SYNTH_WRITE_ONLY for o in ops]
        return r

    @staticmethod
    def decode(resp, some) -> list:
        return [int(v) for v in resp]

    @staticmethod
    def read_batch(dev: DeviceReplica, ops) -> list:
        a = np.zeros(len(ops), SYNTH_RD_DTYPE)
        a["tid"] = [o.tid for o in ops]
        a["r1"] = [o.r1 for o in ops]
        a["r2"] = [o.r2 for o in ops]
        return [int(x) for x in dev.sy_read(a)]

    @staticmethod
    def snapshot(dev: DeviceReplica):
        return dev.sy_dump()


# =====================================================================================
# Log / Replica / ReplicaToken — the reference's public API
# =====================================================================================
class ReplicaToken:
    """nr/src/replica.rs:26-48"""

    __slots__ = ("_id",)

    def __init__(self, ident: int):
        self._id = ident

    def id(self) -> int:
        return self._id

    def __eq__(self, o):
        return isinstance(o, ReplicaToken) and o._id == self._id

    def __repr__(self):
        return f"ReplicaToken({self._id})"


class Log:
    """nr::Log — the shared operation log (nr/src/log.rs:88-131).

    Physically, every registered GPU replica holds a copy of the log in its HBM ring; an
    append writes the same records at the same logical indices into every copy (in one
    process the copies are filled directly; across processes/GPUs the write segments are
    all-gathered, see parallel.py). `tail` is the shared logical tail, `ctail` the max tail any
    replica has replayed (nr/src/log.rs:522), used by reads to sync.

    The host keeps the appended batches of the live window [head, tail) (head = the slowest
    replica's ltail, advanced when the log nears full as Log::append's GC does,
    nr/src/log.rs:364-387, :536-580), so that a replica registered after appends can be given the
    entries it has not seen and catch up through exec from its ltail = 0 (nr/src/log.rs:272-292,
    :473-524; nr/src/replica.rs:469-479).
    """

    def __init__(self, nbytes: int = DEFAULT_LOG_BYTES):
        num = nbytes // 64
        if num < 2 * GC_FROM_HEAD:
            num = 2 * GC_FROM_HEAD
        size = 1
        while size < num:
            size <<= 1
        self.bytes = nbytes
        self.size = size
        self.head = 0
        self.tail = 0
        self.ctail = 0
        self._next = 1
        self._replicas: List["Replica"] = []
        self._live: list = []  # (first log index, records, origin) of the batches in [head, tail)
        self.lock = threading.RLock()

    def register(self, replica: "Replica") -> Optional[int]:
        """Log::register (nr/src/log.rs:272-292): ids 1.., None at MAX_REPLICAS. A replica
        registered after appends starts at ltail 0 like the reference's; its copy of the log is
        filled with the live entries, which it replays on its next combine or sync. If GC has
        already moved head past entry 0 the reference's exec would panic ("Local tail not within
        the shared log", nr/src/log.rs:486-488): here registration fails with RuntimeError."""
        with self.lock:
            if self._next >= MAX_REPLICAS:
                return None
            if self.head > 0:
                raise RuntimeError(f"cannot register a replica: the log was garbage-collected up to {self.head}, "
                                   "so entries a new replica must replay from index 0 are gone")
            for first, recs, origin in self._live:  # catch-up copy, same logical indices
                got = replica.dev.log_append(recs, origin)
                if got != first:
                    raise RuntimeError("log copies diverged")
            idx = self._next
            self._next += 1
            self._replicas.append(replica)
            return idx

    def _ltails(self):
        return [r.dev.log_state()["ltail"] for r in self._replicas]

    def get_ctail(self) -> int:
        """Log::get_ctail (nr/src/log.rs:677-679): the largest tail any replica has replayed."""
        with self.lock:
            self.ctail = max([self.ctail] + self._ltails())
            return self.ctail

    def is_replica_synced_for_reads(self, replica: "Replica", ctail: Optional[int] = None) -> bool:
        """Log::is_replica_synced_for_reads (nr/src/log.rs:671-673): ltail >= ctail."""
        c = self.get_ctail() if ctail is None else ctail
        return replica.dev.log_state()["ltail"] >= c

    def advance_head(self) -> int:
        """Log::advance_head (nr/src/log.rs:536-580): head = min over replicas' ltails (each
        device replica's own ring is garbage-collected up to its ltail by libnrgpu.so)."""
        with self.lock:
            lt = self._ltails()
            if lt:
                self.head = max(self.head, min(lt))
            return self.head

    def append(self, recs: np.ndarray, idx: int) -> int:
        """Log::append: the same records at the same logical indices in every copy."""
        with self.lock:
            first = None
            for r in self._replicas:
                f = r.dev.log_append(recs, idx)
                if first is None:
                    first = f
                elif f != first:
                    raise RuntimeError("log copies diverged")
            self.tail = first + len(recs)
            self._live.append((first, np.array(recs, copy=True), idx))
            if self.tail - self.head > self.size - GC_FROM_HEAD:  # nearly full: GC (nr/src/log.rs:364-387)
                self.advance_head()
            while self._live and self._live[0][0] + len(self._live[0][1]) <= self.head:
                self._live.pop(0)
            return first


class Replica:
    """nr::Replica<D> (nr/src/replica.rs:72-595) over a GPU replica backend."""

    def __init__(self, log: Log, ds, device: int = 0, **cfg):
        self.ds = ds
        self.log = log
        cfg.setdefault("log_bytes", log.bytes)
        self.dev = DeviceReplica(ds.kind, device, **cfg)
        idx = log.register(self)
        if idx is None:
            raise RuntimeError("too many replicas registered with the log")
        self.idx = idx
        self._next = 1
        self._combiner = threading.Lock()
        self._ctx: dict = {}
        self._resp: dict = {}
        self._reg = threading.Lock()
        # a thread's pending ops are appended and taken under this lock (the reference's
        # per-thread context rings, nr/src/context.rs:88-194, are lock-free SPSC queues)
        self._ctx_lock = threading.Lock()

    # register (nr/src/replica.rs:279-298): tokens 1..=MAX_THREADS_PER_REPLICA
    def register(self) -> Optional[ReplicaToken]:
        with self._reg:
            if self._next > MAX_THREADS_PER_REPLICA:
                return None
            t = self._next
            self._next += 1
            with self._ctx_lock:
                self._ctx[t] = []
                self._resp[t] = []
            return ReplicaToken(t)

    def _enqueue(self, ops, tid):
        with self._ctx_lock:
            q = self._ctx[tid]
            if len(q) + len(ops) > MAX_PENDING_OPS and len(ops) <= MAX_PENDING_OPS:
                return False
            q.extend(ops)
            return True

    def _combine(self):
        """Replica::combine (nr/src/replica.rs:544-595): collect every thread's pending ops,
        append them as one batch, replay the log, route this replica's responses back."""
        with self.log.lock:
            order, batch = [], []
            with self._ctx_lock:
                for t in sorted(self._ctx):
                    q = self._ctx[t]
                    if q:
                        order.append((t, len(q)))
                        batch.extend(q)
                        self._ctx[t] = []
            if batch:
                first = self.log.append(self.ds.encode(batch), self.idx)
                resp, some = self.dev.log_exec(first, first + len(batch))
                out = self.ds.decode(resp, some)
                s = 0
                for t, n in order:
                    self._resp[t].extend(out[s:s + n])
                    s += n
            else:
                self.dev.log_exec()
            st = self.dev.log_state()
            self.log.ctail = max(self.log.ctail, st["ltail"])

    def _combine_until(self, done: Callable[[], bool]):
        """Flat combining's wait (nr/src/replica.rs:508-541): until done(), become the combiner
        and combine every thread's pending ops. The reference spins on a failed try-lock; a
        Python thread spinning on the GIL only lets the combiner run every switch interval
        (5 ms), so a thread blocks on the combiner lock instead and re-checks after it: a
        combine that ran meanwhile may have carried its ops."""
        while not done():
            with self._combiner:
                if not done():
                    self._combine()

    def execute_mut(self, op, tok: ReplicaToken):
        """Replica::execute_mut (nr/src/replica.rs:345-356)"""
        return self.execute_mut_batch([op], tok)[0]

    def execute_mut_batch(self, ops: Sequence, tok: ReplicaToken) -> list:
        """Host batcher: enqueue many of this thread's writes, combine once."""
        tid = tok.id()
        ops = list(ops)
        self._combine_until(lambda: self._enqueue(ops, tid))
        want = len(ops)
        self._combine_until(lambda: len(self._resp[tid]) >= want)
        out = self._resp[tid][:want]
        del self._resp[tid][:want]
        return out

    def _sync_to(self, ctail: int):
        self._combine_until(lambda: self.dev.log_state()["ltail"] >= ctail)

    def execute(self, op, tok: ReplicaToken):
        """Replica::execute -> read_only (nr/src/replica.rs:404-410, :483-497)"""
        return self.execute_batch([op], tok)[0]

    def execute_batch(self, ops: Sequence, tok: ReplicaToken) -> list:
        """Sync to ctail, then dispatch with this replica's replay excluded (the reference's
        reader lock against the combiner, nr/src/replica.rs:483-497). The device answers reads
        only with its copy of the log fully replayed (nrg_hashmap_get: NRG_E_NOT_SYNCED
        otherwise), and other replicas' combiners may append to that copy after the sync: those
        entries -- none of them this replica's own, whose combine appends and replays in one go --
        are replayed first, under the log lock so that no further append lands before the read
        (a read then sees a state at least as new as the ctail it synced to, as NR's does)."""
        self._sync_to(self.log.ctail)
        with self._combiner:
            with self.log.lock:
                self.dev.log_exec()
                return self.ds.read_batch(self.dev, list(ops))

    def sync(self, tok: Optional[ReplicaToken] = None):
        """Replica::sync (nr/src/replica.rs:473-479)"""
        self._sync_to(self.log.ctail)

    def verify(self, v: Callable):
        """Replica::verify (nr/src/replica.rs:443-467): catch up on the log, then run v on
        the replica's data structure (materialised on the host)."""
        with self._combiner:
            with self.log.lock:
                self.dev.log_exec()
                self.dev.sync()
                v(self.ds.snapshot(self.dev))
