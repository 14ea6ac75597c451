"""Phase timings of st_tile_kernel (diagnostic; run on the GPU box).

Opens a stack replica with knob EXP=2 (timestamps), replays rounds of N ops over a
50,000-element stack and prints, per phase, the mean and max over tiles of the time since the
tile's start (wall_clock64, 100 MHz), plus the spread of tile start times.
Usage: python microbench/stack_phases.py [N]
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

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
dev = nrgpu.DeviceReplica(L.NRG_DS_STACK, 0, knobs={"EXP": int(os.environ.get("EXP", "2"), 0)}, max_batch=N, stack_capacity=N * 4 + 100_000, pipeline=int(os.environ.get("PIPE", "1")),
                          log_bytes=64 * 4 * max(N, 8192))
dev.use_torch_stream()
dev.st_init(list(range(50_000)))
# BB=k: k back-to-back rounds over distinct batches before each reading (as bench.py runs them)
BB = int(os.environ.get("BB", "1"))
opsl = [torch.empty(N, dtype=torch.int64, device="cuda") for _ in range(BB)]
for i, o in enumerate(opsl):
    dev.gen_stack_ops_device(o, N, 12345 + i)
resps = [torch.empty(N, dtype=torch.int32, device="cuda") for _ in range(2)]
somes = [torch.empty(N, dtype=torch.uint8, device="cuda") for _ in range(2)]
TILE = int(os.environ.get("ST_TILE", "2048"))  # ops per tile of the build (256 lanes x NRG_ST_OPS)
tiles = (N + TILE - 1) // TILE
names = ["loads", "local pass", "scan+responses", "lookback", "query list+sparse table", "queries", "table"]
acc = np.zeros((tiles, 9))
w0 = []
R = 20
fin = []
q8 = []
lb = []
for r in range(R + 3):
    for i in range(BB):  # pipeline=1: a round's finish rides in the next launch
        dev.st_round_device(opsl[i], N, 1, resps[i & 1], somes[i & 1])
    torch.cuda.synchronize()
    buf = np.zeros(tiles * 16, np.uint64)
    L.check(L.load().nrg_test_debug_read(dev.handle, buf.ctypes.data_as(C.c_void_p), tiles * 16))
    full = np.zeros(256 * 16, np.uint64)
    L.check(L.load().nrg_test_debug_read(dev.handle, full.ctypes.data_as(C.c_void_p), 256 * 16))
    fb = full.reshape(256, 16)[128:128 + tiles, :2].astype(np.float64)
    t = buf.reshape(tiles, 16)[:, :9].astype(np.float64)
    if r >= 3 and fb[:, 0].min() > 0:
        o = min(t[:, 0].min(), fb[:, 0].min())
        fin.append((fb[:, 0].min() - o, fb[:, 0].max() - o, fb[:, 1].max() - o, t[:, 0].min() - o, t[:, 7].max() - o))
    if r >= 3:
        q8.append((t[:, 8] - t[:, 5]).mean() / 100.0)
        t9 = buf.reshape(tiles, 16)[:, 9:11].astype(np.float64)
        w0.append(((t9[:, 0] - t[:, 5]).mean() / 100.0, t9[:, 1].mean(), ((t[:, 6] - t[:, 8]).mean() / 100.0)))
    if r >= 3:
        acc += t - t[:, :1].min()
        x = buf.reshape(tiles, 16).astype(np.float64)
        o = x[:, 0].min()
        pub, built, res, q1 = x[:, 15] - o, x[:, 12] - o, x[:, 13] - o, x[:, 14] - o
        mpred = np.maximum.accumulate(np.concatenate([[0.0], pub[:-1]]))  # latest predecessor publish
        lb.append(np.array([(pub - (x[:, 0] - o)).mean(), (built - pub).mean(), (res - built).mean(),
                            (res - np.maximum(mpred, built)).mean(), pub.max(), np.argmax(pub),
                            (q1 - built).mean(), (res - built).max()]))
acc /= R
start = acc[:, 0]
print(f"N={N} tiles={tiles}: tile start spread {start.min() / 100:.2f}..{start.max() / 100:.2f} us")
for k, nm in enumerate(names):
    d = (acc[:, k + 1] - acc[:, k]) / 100.0
    print(f"  {nm:14s} mean {d.mean():7.2f} us  max {d.max():7.2f} us")
end = acc[:, 7] / 100.0
print(f"  last tile end {end.max():.2f} us after the first start; mean tile span {(acc[:, 7] - acc[:, 0]).mean() / 100:.2f} us")
if fin:
    f = np.array(fin).mean(0) / 100.0
    print("fused finish of the previous chunk (us from the launch's first workgroup): start %.2f..%.2f, last end %.2f;"
          " tiles start %.2f, last tile end %.2f" % tuple(f))
hw = buf.reshape(tiles, 16)[:, 11]
cu = [(int(h) >> 32 & 15, int(h) >> 13 & 3, int(h) >> 12 & 1, int(h) >> 8 & 15) for h in hw]  # xcc, se, sh, cu
from collections import Counter
cnt = Counter(cu)
share = np.array([cnt[c] for c in cu])
ld = (acc[:, 1] - acc[:, 0]) / 100.0
print("  placement (last round): %d tiles on %d CUs; tiles sharing a CU: %d; load mean %.2f us alone, %.2f us shared"
      % (tiles, len(cnt), int((share > 1).sum()), ld[share == 1].mean() if (share == 1).any() else 0, ld[share > 1].mean() if (share > 1).any() else 0))
slow = np.argsort(-ld)[:8]
print("  slowest loads: " + ", ".join("tile %d %.2f us (xcc %d se %d cu %d, %d on CU)" % (k, ld[k], cu[k][0], cu[k][1], cu[k][3], share[k]) for k in slow))
if q8:
    print("  of the unmatched-Pop phase, the intra-tile queries: mean %.2f us" % np.mean(q8))
    print("  wave 0's own queries %.2f us over a list of %.0f; pre-chunk pass %.2f us" % tuple(np.mean(w0, 0)))
if lb:
    v = np.mean(lb, 0) / np.array([100, 100, 100, 100, 100, 1, 100, 100])
    print("  publish %.2f us after the tile's start; publish -> query structures built %.2f; wave 0's wait %.2f"
          " (max %.2f), of it after the latest predecessor's publish (or the build) %.2f; latest publish at %.2f us"
          " (tile ~%.0f); wave 1's queries %.2f" % (v[0], v[1], v[2], v[7], v[3], v[4], v[5], v[6]))
