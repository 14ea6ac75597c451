"""Phase timings of hm_papply_kernel, the partition rounds' apply (diagnostic; run on the GPU box).

Opens a hashmap replica as bench.py does (2^26 slots, prefill [0, 2^23) -> k+1, uniform keys over
10M) with knob EXP=2 (timestamps), replays pipelined rounds of W Puts + R Gets and prints, per
phase, the mean and max over buckets (wall_clock64, 100 MHz = 10 ns ticks) of:
  counts   start -> the bucket's [tile][bucket] counts gathered and scanned
  hash     -> the first chunk's tile map built, its entries landed and hashed by key
  resolve  -> its keys' slots found or claimed (pa_resolve: probe lines, CAS on empty slots)
  store    -> its values stored, hash entries freed
  rest     -> the remaining chunks
and the spread of workgroup starts and ends. Usage:
  python microbench/papply_phases.py W R [PA_TPB]     (e.g. 800000 900000 1024)
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

W = int(sys.argv[1]) if len(sys.argv) > 1 else 800_000
R = int(sys.argv[2]) if len(sys.argv) > 2 else 900_000
TPB = int(sys.argv[3]) if len(sys.argv) > 3 else 0
knobs = {"EXP": 2, "PART": 2}
if TPB:
    knobs["PA_TPB"] = TPB
dev = nrgpu.DeviceReplica(L.NRG_DS_HASHMAP, 0, knobs=knobs, log2_slots=26, max_batch=max(W, 8192),
                          max_reads=max(R, 8192), log_bytes=64 * 4 * max(W, 8192), pipeline=1)
dev.use_torch_stream()
dev.hm_prefill_range(1 << 23, 1)
g = torch.Generator(device="cuda")
g.manual_seed(11)
rounds, warm = 12, 3
NBMAX = 1024
acc = np.zeros(7)
mx = np.zeros(7)
cnt = 0
for r in range(rounds + warm):
    puts = torch.empty((W, 2), dtype=torch.int64, device="cuda")
    puts[:, 0] = torch.randint(0, 10_000_000, (W,), generator=g, device="cuda")
    puts[:, 1] = torch.randint(-(1 << 62), 1 << 62, (W,), generator=g, device="cuda")
    gk = torch.randint(0, 10_000_000, (R,), generator=g, device="cuda")
    gv = torch.empty(R, dtype=torch.int64, device="cuda")
    gf = torch.empty(R, dtype=torch.uint8, device="cuda")
    dev.hm_round_device(puts, W, 1, gk, R, gv, gf, None, None)
    torch.cuda.synchronize()  # this round's apply ran (its reads are deferred to the next round)
    buf = np.zeros(NBMAX * 8, np.uint64)
    L.check(L.load().nrg_test_debug_read(dev.handle, buf.ctypes.data_as(C.c_void_p), buf.size))
    rows = buf.reshape(NBMAX, 8).astype(np.float64)
    rows = rows[rows[:, 0] > 0]
    if r < warm or len(rows) == 0:
        continue
    t0 = rows[:, 0].min()
    d = np.stack([rows[:, 0] - t0,                      # start offset
                  rows[:, 1] - rows[:, 0],              # counts
                  rows[:, 2] - rows[:, 1],              # hash (first chunk)
                  rows[:, 3] - rows[:, 2],              # resolve (first chunk)
                  rows[:, 4] - rows[:, 3],              # store (first chunk)
                  rows[:, 5] - rows[:, 4],              # rest
                  rows[:, 5] - t0], axis=1) / 100.0     # end offset; ticks -> us
    acc += d.mean(axis=0)
    mx += d.max(axis=0)
    cnt += 1
    nb, chunks = len(rows), rows[:, 6].mean()
dev.join()
names = ["start", "counts", "hash", "resolve", "store", "rest", "end"]
print(f"hm_papply phases: W={W} R={R} PA_TPB={TPB or 'default'}: {nb} buckets, {chunks:.2f} chunks each, {cnt} rounds")
print("           " + " ".join(f"{n:>9s}" for n in names))
print("mean (us)  " + " ".join(f"{v:9.2f}" for v in acc / cnt))
print("max  (us)  " + " ".join(f"{v:9.2f}" for v in mx / cnt))
