"""Phase timings of hm_elect_kernel<true> on B1 rounds with previous values (diagnostic; GPU box).

Opens the B1 replica (2^26 slots, prefill 2^23, keys over 10M), replays rounds of 100k Puts +
900k Gets asking for previous values, with knob EXP=65536 (elector timestamps, wall_clock64 at
100 MHz), and prints per phase the mean and max over buckets.
Usage: python microbench/elect_phases.py
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "node-replication_amd"))
import nrgpu  # noqa: E402
from nrgpu import _lib as L  # noqa: E402

W, R = 100_000, 900_000
dev = nrgpu.DeviceReplica(L.NRG_DS_HASHMAP, 0, knobs={"EXP": 0x10000}, log2_slots=26, max_batch=W, log_bytes=64 * 4 * W)
dev.use_torch_stream()
dev.hm_prefill_range(1 << 23, 1)
P = 8
puts = torch.empty((P, W, 2), dtype=torch.int64, device="cuda")
gk = torch.empty((P, R), dtype=torch.int64, device="cuda")
tk = torch.empty(W, dtype=torch.int64, device="cuda")
tv = torch.empty(W, dtype=torch.int64, device="cuda")
for p in range(P):
    dev.gen_uniform_device(tk, W, 1000 + 3 * p, 10_000_000)
    dev.gen_raw_device(tv, W, 1001 + 3 * p)
    dev.gen_puts_device(puts[p], tk, tv, W)
    dev.gen_uniform_device(gk[p], R, 1002 + 3 * p, 10_000_000)
gv = torch.empty(R, dtype=torch.int64, device="cuda")
gf = torch.empty(R, dtype=torch.uint8, device="cuda")
pv = torch.empty(W, dtype=torch.int64, device="cuda")
pf = torch.empty(W, dtype=torch.uint8, device="cuda")
NB = 512
names = ["count row + scan", "pass 1 (gather + hash)", "claims + old values", "walk", "stores + end"]
acc = np.zeros((NB, 7))
n = 0
for r in range(24):
    dev.hm_round_device(puts[r % P], W, 1, gk[r % P], R, gv, gf, pv, pf)
    dev.join()
    torch.cuda.synchronize()
    if r < 4:
        continue
    buf = np.zeros(NB * 16, np.uint64)
    L.check(L.load().nrg_test_debug_read(dev.handle, buf.ctypes.data_as(C.c_void_p), NB * 16))
    t = buf.reshape(NB, 16)[:, :7].astype(np.float64)
    t0 = t[:, 0].min()
    t[:, :6] -= t0
    acc += t
    n += 1
acc /= n
print(f"buckets={NB} entries/bucket mean {acc[:, 6].mean():.0f} max {acc[:, 6].max():.0f}; "
      f"start spread {acc[:, 0].min() / 100:.2f}..{acc[:, 0].max() / 100:.2f} us")
for k, nm in enumerate(names):
    d = (acc[:, k + 1] - acc[:, k]) / 100.0
    print(f"  {nm:24s} mean {d.mean():7.2f} us  max {d.max():7.2f} us")
print(f"  last bucket end {acc[:, 5].max() / 100:.2f} us; mean span {(acc[:, 5] - acc[:, 0]).mean() / 100:.2f} us")
