"""Multi-GPU node replication: one replica per GPU, one process per GPU.

In NR every replica replays every write (nr/src/log.rs:473-524, one exec loop per replica
over the shared log); the reference shares the log through cache-coherent memory across
NUMA nodes. Here each GPU is a NUMA node: per round, every rank contributes the write segment
its clients produced, the segments are all-gathered, and every replica replays the identical
global log W_0 || W_1 || ... || W_{G-1} (concatenation by rank = the deterministic log order
of the round), then answers its own reads against the post-round state. Responses to writes go
only to the origin rank (nr/src/replica.rs:576-578). Reads never leave their GPU.

Two transports, one round semantics:
  ReplicaGroup      the C ABI's group (nrg_group_join / nrg_group_round_async): RCCL over xGMI,
                    called from libnrgpu.so on a library-owned stream per GPU, all-gather of
                    round e+1 overlapping the replay of round e. The MI355X path.
  ReplicatedLog /   the same rounds with the all-gather done by torch.distributed (gloo), for
  ReplicatedHashMap multi-process tests on hosts without GPUs-per-rank (CPU `gloo` tests, the
                    1-GPU box rehearsal); the replay is the same C-ABI call
                    (nrg_hashmap_round_segments_async / append_segments + exec).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import torch
import torch.distributed as dist

from . import _lib as L


def _ptr(t) -> int:
    if t is None:
        return 0
    return t if isinstance(t, int) else t.data_ptr()


class ReplicaGroup:
    """This process's replica as one member of a libnrgpu.so replica group (RCCL).

    The group id (ncclUniqueId) is created by rank 0 and broadcast over the default
    torch.distributed process group; every rank then joins with its own replica
    (nrg_group_join, ncclCommInitRank on the replica's GPU), which blocks until every rank has
    joined. A caller that ships the id itself (`uid`, from unique_id()) needs no process group:
    tests run one thread per rank over the loopback collectives that way."""

    @staticmethod
    def unique_id() -> bytes:
        """nrg_group_unique_id (ncclGetUniqueId, or a loopback id while those are selected)."""
        uid = (C.c_uint8 * L.NRG_GROUP_ID_BYTES)()
        L.check(L.load().nrg_group_unique_id(uid), "nrg_group_unique_id")
        return bytes(uid)

    def __init__(self, replica, rank: Optional[int] = None, world: Optional[int] = None,
                 pg: Optional[dist.ProcessGroup] = None, uid: Optional[bytes] = None,
                 timeout_ms: Optional[int] = None):
        lib = L.load()
        self.replica = replica
        self.rank = dist.get_rank(pg) if rank is None else rank
        self.world = dist.get_world_size(pg) if world is None else world
        if uid is not None:
            uid = (C.c_uint8 * L.NRG_GROUP_ID_BYTES).from_buffer_copy(uid)
        else:
            uid = (C.c_uint8 * L.NRG_GROUP_ID_BYTES)()
            if self.rank == 0:
                L.check(lib.nrg_group_unique_id(uid), "nrg_group_unique_id")
            if self.world > 1:
                obj = [bytes(uid)]
                dist.broadcast_object_list(obj, src=0, group=pg)
                uid = (C.c_uint8 * L.NRG_GROUP_ID_BYTES).from_buffer_copy(obj[0])
        h = C.c_void_p()
        L.check(lib.nrg_group_join(replica.handle, uid, self.world, self.rank, C.byref(h)), "nrg_group_join")
        self._h = h
        self._lib = lib
        if timeout_ms is not None:
            self.set_timeout(timeout_ms)
        self._round = L.Round()
        self._lens = None

    def set_timeout(self, ms: int):
        """nrg_group_set_timeout: deadline of every wait on the peer ranks. A round or sync whose
        peers miss it raises NrgError(NRG_E_TIMEOUT) naming this rank and round."""
        L.check(self._lib.nrg_group_set_timeout(self._h, int(ms)), "nrg_group_set_timeout")

    def last_error(self) -> str:
        """nrg_group_last_error: the group's sticky failure, '' if none."""
        return (self._lib.nrg_group_last_error(self._h) or b"").decode()

    def _check(self, rc: int, what: str):
        if rc:
            diag = self.last_error()
            L.check(rc, f"{what} [{diag}]" if diag else what)

    def set_input_stream(self, stream_ptr: int):
        """All-gathers wait only for work on this stream (where the inputs are produced)."""
        L.check(self._lib.nrg_group_set_input_stream(self._h, 0, C.c_void_p(stream_ptr)))

    def round_async(self, recs, n: int, resp=None, some=None, get_keys=None, n_gets: int = 0, get_vals=None,
                    get_found=None, seg_lens: Optional[Sequence[int]] = None):
        """One NR round (device tensors or raw pointers): all-gather + replay + local reads.

        seg_lens: every rank's segment length, the same list on every rank (the stream-ordered
        path; a header checks it on every rank). None: the lengths are exchanged first, which
        costs one host round trip but lets every rank's n differ."""
        r = self._round
        r.recs, r.n, r.resp, r.some = _ptr(recs), n, _ptr(resp), _ptr(some)
        r.get_keys, r.n_gets, r.get_vals, r.get_found = _ptr(get_keys), n_gets, _ptr(get_vals), _ptr(get_found)
        lens = None
        if seg_lens is not None:
            if self._lens is None or list(self._lens) != list(seg_lens):
                self._lens = (C.c_uint64 * self.world)(*seg_lens)
            lens = self._lens
        rc = self._lib.nrg_group_round_async(self._h, C.byref(r), lens)
        if rc:
            self._check(rc, "nrg_group_round_async")

    def sync(self):
        self._check(self._lib.nrg_group_sync(self._h), "nrg_group_sync")

    def close(self):
        if getattr(self, "_h", None):
            self._lib.nrg_group_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class Gathered:
    """One round's all-gathered write log (in flight until wait())."""

    __slots__ = ("buf", "work", "stride", "lens", "words")

    def __init__(self, buf, work, stride, lens, words):
        self.buf, self.work, self.stride, self.lens, self.words = buf, work, stride, lens, words

    def wait(self):
        if self.work is not None:
            self.work.wait()
            self.work = None


class ReplicatedLog:
    """One replica per rank of any NR data structure, driven in rounds of write segments, with
    the all-gather done by torch.distributed (gloo; see ReplicaGroup for RCCL).

    round() = gather_async() + replay(). Records are int64 tensors [W, words] (words = record
    bytes / 8: hashmap 2, stack 1, synthetic 4)."""

    NBUF = 3  # gathered-log buffers in rotation

    def __init__(self, replica, group: Optional[dist.ProcessGroup] = None, device: Optional[torch.device] = None):
        self.replica = replica
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device if device is not None else torch.device("cpu")
        self.origins = [r + 1 for r in range(self.world)]  # replica ids start at 1 (nr/src/log.rs:272-292)
        self._bufs = [None] * self.NBUF
        self._next = 0

    def _buf(self, need: int) -> torch.Tensor:
        i = self._next
        self._next = (i + 1) % self.NBUF
        b = self._bufs[i]
        if b is None or b.numel() < need:
            b = torch.empty(need, dtype=torch.int64)
            self._bufs[i] = b
        return b[:need]

    def exchange_lengths(self, W: int):
        t = torch.tensor([W], dtype=torch.int64)
        out = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [int(x.item()) for x in out]

    def gather_async(self, recs: torch.Tensor, stride: Optional[int] = None, lens=None) -> Gathered:
        """All-gather this rank's write segment (records in issue order). Fixed-size rounds pass
        `stride` (segment capacity) and skip the length exchange."""
        if recs.dim() == 1:
            recs = recs.reshape(-1, 1)
        W, words = recs.shape
        if lens is None:
            lens = [W] * self.world if stride is not None else self.exchange_lengths(W)
        if stride is None:
            stride = max(lens) if lens else 0
        seg = torch.zeros((stride, words), dtype=torch.int64)
        seg[:W] = recs.cpu()
        out = self._buf(self.world * stride * words)
        dist.all_gather_into_tensor(out, seg.reshape(-1), group=self.group)
        return Gathered(out.to(recs.device), None, stride, lens, words)

    def replay(self, g: Gathered, resp: Optional[torch.Tensor] = None, some: Optional[torch.Tensor] = None):
        """Log::append of the gathered segments in rank order (the round's global log order),
        then Log::exec; responses only for this rank's own segment (nr/src/replica.rs:576-578)."""
        g.wait()
        firsts = self.replica.log_append_segments(g.buf, g.stride, g.lens, self.origins)
        lo = firsts[self.rank]
        self.replica.log_exec_device(lo, lo + g.lens[self.rank], resp, some)

    def round(self, recs: torch.Tensor, resp=None, some=None, stride: Optional[int] = None, lens=None):
        g = self.gather_async(recs, stride, lens)
        self.replay(g, resp, some)
        return g.buf


class ReplicatedHashMap(ReplicatedLog):
    """NrHashMap replicas: a round is (write segment, local reads); the fused device round
    appends, replays and answers the reads against the post-round state."""

    def replay(self, g: Gathered, get_keys: torch.Tensor, get_vals: torch.Tensor, get_found: torch.Tensor,
               prev: Optional[torch.Tensor] = None, prev_found: Optional[torch.Tensor] = None):
        """Append the gathered segments in rank order, replay them, answer this rank's reads
        against the post-round state; Put responses (prev) only for this rank's own segment."""
        g.wait()
        self.replica.hm_round_segments_device(g.buf, g.stride, g.lens, self.origins, self.rank, get_keys,
                                              get_keys.shape[0], get_vals, get_found, prev, prev_found)

    def round(self, puts: torch.Tensor, get_keys: torch.Tensor, get_vals: torch.Tensor, get_found: torch.Tensor,
              prev: Optional[torch.Tensor] = None, prev_found: Optional[torch.Tensor] = None,
              stride: Optional[int] = None, lens=None):
        """One NR round: puts [W, 2] int64 (key, value) on this rank's device, in issue order."""
        g = self.gather_async(puts, stride, lens)
        self.replay(g, get_keys, get_vals, get_found, prev, prev_found)
        return g.buf.view(-1, 2)


# ---- cnr-style key-partitioned NrHashMap ----------------------------------
# cnr maps every operation to one of several logs with LogMapper::hash (cnr/src/lib.rs:134-167,
# cnr/src/replica.rs:430-445) and each log replays on its own (:673-736). Here partition p's log
# lives on rank p, which holds only the keys it owns: a round routes Puts and Gets to their
# owners, every owner replays what it received in rank order (for each key the NR global-log
# order) and answers its Gets, and the answers come back in the caller's order. Answers equal
# NR's; the replicas hold one partition each (their digests add up to the NR replica's).

_M1, _M2 = 0xBF58476D1CE4E5B9, 0x94D049BB133111EB


def key_owner(keys, parts: int):
    """nrg_key_owner over an array: (low 32 bits of splitmix64(key)) * parts >> 32."""
    import numpy as np

    z = np.ascontiguousarray(keys).view(np.uint64).copy()
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(_M1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(_M2)
        z = z ^ (z >> np.uint64(31))
    return ((z & np.uint64(0xFFFFFFFF)) * np.uint64(parts) >> np.uint64(32)).astype(np.int64)


class PartitionedGroup(ReplicaGroup):
    """This rank's replica as partition `rank` of a key-partitioned group (libnrgpu.so, RCCL
    send/recv): nrg_group_partitioned_round."""

    def round(self, puts, n: int, get_keys, n_gets: int, get_vals, get_found, prev=None, prev_found=None):
        """One round, queued once its counts are exchanged (nrg_group_partitioned_round)."""
        r = self._round
        r.recs, r.n, r.resp, r.some = _ptr(puts), n, _ptr(prev), _ptr(prev_found)
        r.get_keys, r.n_gets, r.get_vals, r.get_found = _ptr(get_keys), n_gets, _ptr(get_vals), _ptr(get_found)
        rc = self._lib.nrg_group_partitioned_round(self._h, C.byref(r))
        if rc:
            self._check(rc, "nrg_group_partitioned_round")

    def round_async(self, puts, n: int, get_keys, n_gets: int, get_vals, get_found, prev=None, prev_found=None):
        """Pipelined: queue this round, move the previous one to its owners and replay it, and send
        the one before back (nrg_group_partitioned_round_async). A round's buffers stay borrowed
        for the next two round_async calls, or until flush / sync."""
        r = self._round
        r.recs, r.n, r.resp, r.some = _ptr(puts), n, _ptr(prev), _ptr(prev_found)
        r.get_keys, r.n_gets, r.get_vals, r.get_found = _ptr(get_keys), n_gets, _ptr(get_vals), _ptr(get_found)
        rc = self._lib.nrg_group_partitioned_round_async(self._h, C.byref(r))
        if rc:
            self._check(rc, "nrg_group_partitioned_round_async (the previous round)")

    def flush(self):
        """Complete the round queued by round_async, if any."""
        rc = self._lib.nrg_group_partitioned_flush(self._h)
        if rc:
            self._check(rc, "nrg_group_partitioned_flush")


class PartitionedHashMap:
    """Key-partitioned rounds with the exchanges done by torch.distributed (all_to_all_single;
    gloo on CPU tests, see PartitionedGroup for RCCL). `replica` must provide
    partitioned_replay(puts [p, 2] int64, keys [k] int64, want_prev) -> (vals, found, prev, prev_found)
    (DeviceReplica does; CPU tests use an oracle-backed double)."""

    def __init__(self, replica, group: Optional[dist.ProcessGroup] = None):
        self.replica = replica
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def _split(self, keys: torch.Tensor):
        """Stable partition by owner: (order, counts); order[j] = index of the j-th routed item."""
        import numpy as np

        own = key_owner(keys.cpu().numpy(), self.world)
        order = np.argsort(own, kind="stable")
        counts = np.bincount(own, minlength=self.world)
        return torch.from_numpy(order), [int(c) for c in counts]

    def _a2a(self, send: torch.Tensor, send_counts, recv_counts):
        out = torch.empty((sum(recv_counts),) + tuple(send.shape[1:]), dtype=send.dtype)
        dist.all_to_all_single(out, send.contiguous(), [c for c in recv_counts], [c for c in send_counts],
                               group=self.group)
        return out

    def round(self, puts: torch.Tensor, get_keys: torch.Tensor, get_vals: torch.Tensor, get_found: torch.Tensor,
              prev: Optional[torch.Tensor] = None, prev_found: Optional[torch.Tensor] = None):
        """puts [W, 2] int64 (key, value) and get_keys [R] in issue order, on any device; answers
        land in get_vals / get_found (and prev / prev_found) in that order."""
        dev = get_vals.device
        p_cpu, k_cpu = puts.reshape(-1, 2).cpu(), get_keys.reshape(-1).cpu()
        p_order, p_cnt = self._split(p_cpu[:, 0])
        k_order, k_cnt = self._split(k_cpu)
        want = torch.tensor([1 if prev is not None else 0], dtype=torch.int64)
        sizes = torch.tensor(p_cnt + k_cnt + [int(want.item())], dtype=torch.int64)
        allsz = [torch.zeros_like(sizes) for _ in range(self.world)]
        dist.all_gather(allsz, sizes, group=self.group)  # every rank's counts (and wants-prev flag)
        w = self.world
        p_from = [int(allsz[s][self.rank]) for s in range(w)]
        k_from = [int(allsz[s][w + self.rank]) for s in range(w)]
        any_prev = any(int(allsz[s][2 * w]) for s in range(w))
        rput = self._a2a(p_cpu[p_order], p_cnt, p_from)      # received in rank order = log order
        rkey = self._a2a(k_cpu[k_order], k_cnt, k_from)
        vals, found, pv, pf = self.replica.partitioned_replay(rput, rkey, any_prev)
        a_vals = self._a2a(vals.cpu(), k_from, k_cnt)
        a_found = self._a2a(found.cpu(), k_from, k_cnt)
        back_v = torch.empty_like(a_vals)
        back_f = torch.empty_like(a_found)
        back_v[k_order] = a_vals
        back_f[k_order] = a_found
        get_vals.copy_(back_v.to(dev))
        get_found.copy_(back_f.to(dev))
        if any_prev:
            a_pv = self._a2a(pv.cpu(), p_from, p_cnt)
            a_pf = self._a2a(pf.cpu(), p_from, p_cnt)
            if prev is not None:
                bv, bf = torch.empty_like(a_pv), torch.empty_like(a_pf)
                bv[p_order] = a_pv
                bf[p_order] = a_pf
                prev.copy_(bv.to(prev.device))
                prev_found.copy_(bf.to(prev_found.device))
