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


class ReplicatedHashMap:
    """Drives one NrHashMap replica per rank through rounds of (write segment, reads)."""

    def __init__(self, replica, group: Optional[dist.ProcessGroup] = None, device: Optional[torch.device] = None):
        self.replica = replica
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device if device is not None else torch.device("cpu")
        self.backend = dist.get_backend(group)
        self._buf = None

    def _gather(self, seg: torch.Tensor, stride: int) -> torch.Tensor:
        """All-gather fixed-stride segments ([stride, 2] int64 each) into [world*stride, 2]."""
        need = self.world * stride * 2
        if self._buf is None or self._buf.numel() < need or self._buf.device != seg.device:
            self._buf = torch.empty(need, dtype=torch.int64, device=seg.device)
        out = self._buf[:need]
        dist.all_gather_into_tensor(out, seg.reshape(-1), group=self.group)
        return out.view(self.world * stride, 2)

    def exchange_lengths(self, W: int):
        t = torch.tensor([W], dtype=torch.int64, device=self.device if self.backend == "nccl" else "cpu")
        out = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [int(x.item()) for x in out]

    def round(self, puts: torch.Tensor, get_keys: torch.Tensor, get_vals: torch.Tensor, get_found: torch.Tensor,
              prev: Optional[torch.Tensor] = None, prev_found: Optional[torch.Tensor] = None,
              stride: Optional[int] = None, lens=None):
        """One NR round.

        puts: [W, 2] int64 (key, value) on this rank's device, in this rank's issue order.
        stride: segment capacity (fixed-size rounds skip the length exchange); lens: the
        per-rank segment lengths if already known.
        """
        W = puts.shape[0]
        if lens is None:
            lens = [W] * self.world if stride is not None else self.exchange_lengths(W)
        if stride is None:
            stride = max(lens) if lens else 0
        seg = puts
        if W < stride:
            seg = torch.zeros((stride, 2), dtype=torch.int64, device=puts.device)
            seg[:W] = puts
        if self.backend == "gloo" and seg.device.type != "cpu":
            gathered = self._gather(seg.cpu(), stride).to(seg.device)
        else:
            gathered = self._gather(seg.contiguous(), stride)
        origins = [r + 1 for r in range(self.world)]  # replica ids start at 1 (nr/src/log.rs:272-292)
        self.replica.hm_round_segments_device(gathered, stride, lens, origins, self.rank, get_keys,
                                              get_keys.shape[0], get_vals, get_found, prev, prev_found)
        return gathered
