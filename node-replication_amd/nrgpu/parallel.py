"""Multi-GPU node replication: one replica per GPU, one process per GPU.

In NR every replica replays every write (nr/src/log.rs:473-524, one exec loop per replica
over the shared log); the reference shares the log through cache-coherent memory across
NUMA nodes. Here each GPU is a NUMA node: per round, every rank contributes the write segment
its clients produced, the segments are all-gathered (torch.distributed all_gather_into_tensor,
i.e. RCCL over xGMI with the "nccl" backend), and every replica replays the identical global
log W_0 || W_1 || ... || W_{G-1} (concatenation by rank = the deterministic log order of the
round), then answers its own reads against the post-round state. Responses to writes go only
to the origin rank (nr/src/replica.rs:576-578). Reads never leave their GPU.

The exchange is the only collective on the path; it is backend-agnostic so the
host logic runs under `gloo` on CPU (tests) and `nccl` (RCCL) on MI355X.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist


class Gathered:
    """One round's all-gathered write log (in flight until wait())."""

    __slots__ = ("buf", "work", "stride", "lens", "words")

    def __init__(self, buf, work, stride, lens, words):
        self.buf, self.work, self.stride, self.lens, self.words = buf, work, stride, lens, words

    def wait(self):
        if self.work is not None:
            self.work.wait()  # nccl: the current stream waits for the collective (host does not block)
            self.work = None


class ReplicatedLog:
    """One replica per rank of any NR data structure, driven in rounds of write segments.

    round() = gather_async() + replay(). Callers that know the next round's writes early call
    gather_async(next) before replay(current): the all-gather of round e+1 then runs on the
    collective stream while round e replays (the replica's kernels copy the gathered records
    into their own log ring, so a gathered buffer is free once its replay was enqueued; torch's
    ProcessGroupNCCL orders each collective after the work already on the current stream).
    Records are int64 tensors [W, words] (words = record bytes / 8: hashmap 2, stack 1).
    """

    NBUF = 3  # gathered-log buffers in rotation

    def __init__(self, replica, group: Optional[dist.ProcessGroup] = None, device: Optional[torch.device] = None):
        self.replica = replica
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device if device is not None else torch.device("cpu")
        self.backend = dist.get_backend(group)
        self.origins = [r + 1 for r in range(self.world)]  # replica ids start at 1 (nr/src/log.rs:272-292)
        self._bufs = [None] * self.NBUF
        self._next = 0

    def _buf(self, need: int, device) -> torch.Tensor:
        i = self._next
        self._next = (i + 1) % self.NBUF
        b = self._bufs[i]
        if b is None or b.numel() < need or b.device != device:
            b = torch.empty(need, dtype=torch.int64, device=device)
            self._bufs[i] = b
        return b[:need]

    def exchange_lengths(self, W: int):
        t = torch.tensor([W], dtype=torch.int64, device=self.device if self.backend == "nccl" else "cpu")
        out = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [int(x.item()) for x in out]

    def gather_async(self, recs: torch.Tensor, stride: Optional[int] = None, lens=None) -> Gathered:
        """Start the all-gather of this rank's write segment (records in issue order). Fixed-size
        rounds pass `stride` (segment capacity) and skip the length exchange."""
        if recs.dim() == 1:
            recs = recs.reshape(-1, 1)
        W, words = recs.shape
        if lens is None:
            lens = [W] * self.world if stride is not None else self.exchange_lengths(W)
        if stride is None:
            stride = max(lens) if lens else 0
        seg = recs
        if W < stride:
            seg = torch.zeros((stride, words), dtype=torch.int64, device=recs.device)
            seg[:W] = recs
        seg = seg.reshape(-1)
        need = self.world * stride * words
        if self.backend == "gloo" and seg.device.type != "cpu":
            out = self._buf(need, torch.device("cpu"))
            dist.all_gather_into_tensor(out, seg.cpu(), group=self.group)
            return Gathered(out.to(seg.device), None, stride, lens, words)
        out = self._buf(need, seg.device)
        work = dist.all_gather_into_tensor(out, seg.contiguous(), group=self.group, async_op=True)
        return Gathered(out, work, stride, lens, words)

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
