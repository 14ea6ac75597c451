"""Phase timings of sy_bucket_kernel (diagnostic; run on the GPU box).

Opens a synthetic replica as bench.py does (200,000 words, 1 hot + 5 cold touches per ReadWrite)
with knob EXP=2 (timestamps), replays rounds of N ops and prints, per phase, the mean and max over
buckets (wall_clock64, 100 MHz). Usage: python microbench/synth_phases.py [N]
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
dev = nrgpu.DeviceReplica(L.NRG_DS_SYNTHETIC, 0, knobs={"EXP": 2}, max_batch=N, log_bytes=64 * 4 * max(N, 8192),
                           pipeline=1)  # as bench.py: the sums of round e-1 ride in round e's partition launch
dev.use_torch_stream()
g = torch.Generator(device="cuda")
g.manual_seed(7)
ops = torch.empty((N, 4), dtype=torch.int64, device="cuda")
ops[:, 0] = torch.randint(0, 64, (N,), generator=g, device="cuda")
ops[:, 1] = torch.randint(-(1 << 63), (1 << 63) - 1, (N,), generator=g, device="cuda")
ops[:, 2] = torch.randint(-(1 << 63), (1 << 63) - 1, (N,), generator=g, device="cuda")
ops[:, 3] = 1
resp = torch.empty(N, dtype=torch.int64, device="cuda")
some = torch.empty(N, dtype=torch.uint8, device="cuda")
SPAN = 200_000 - 2  # hot_reads = 2
W = -(-(SPAN - 1) // 508)  # synthetic.hip SY_MAX_NB - SY_B0_PARTS
NB = 1 + -(-(SPAN - 1) // W) + 3  # workgroups: bucket 0 (cold word 0) in 4 parts, then the buckets
R = 20
acc = np.zeros((NB, 9))
T = -(-N // 2048)  # partition tiles (synthetic.hip SYA_OPS)
pacc = np.zeros((T, 5))
sacc = np.zeros((T, 3))
hw = None
for r in range(R + 3):
    # two rounds back to back, the second's stamps read: its partition launch follows the first
    # round's bucket pass on a busy queue, as in the bench (a launch from an idle GPU starts its
    # XCDs up to 3 us apart)
    for _ in range(2):
        if os.environ.get("SY_NORESP"):  # (diagnostic: no responses -> the sum role only folds the hot words)
            dev.sy_round_device(ops, N, 1)
        else:
            dev.sy_round_device(ops, N, 1, resp, some)
    torch.cuda.synchronize()
    buf = np.zeros(3072 * 16, np.uint64)  # synthetic.hip SY_DBG_ROWS
    L.check(L.load().nrg_test_debug_read(dev.handle, buf.ctypes.data_as(C.c_void_p), buf.size))
    rows = buf.reshape(3072, 16)
    t = rows[:NB, :9].astype(np.float64)
    pt = rows[1024:1024 + T, :5].astype(np.float64)  # this round's partition tiles
    st = rows[2048:2048 + T, :3].astype(np.float64)  # the previous round's sums (same launch)
    t0 = pt[:, 0].min()  # the round's launch starts with the partition
    for k in (0, 1, 2, 7):
        t[:, k] -= t0
    pt -= t0
    st -= t0
    if r >= 3:
        acc += t
        pacc += pt
        sacc += st
    if r == R + 2:
        hw = rows[:NB, 9:12].astype(np.int64)
        phw = rows[1024:1024 + T, 9:11].astype(np.int64)  # the tiles' HW_ID, XCC_ID
acc /= R
pacc /= R
sacc /= R
print(f"partition tiles {T}: start {pacc[:, 0].min() / 100:.2f}..{pacc[:, 0].max() / 100:.2f} us, last end {pacc[:, 4].max() / 100:.2f} us")
for nm, d in [("load+rank", pacc[:, 1] - pacc[:, 0]), ("offsets", pacc[:, 2] - pacc[:, 1]), ("stage LDS", pacc[:, 3] - pacc[:, 2]),
              ("E stores", pacc[:, 4] - pacc[:, 3]), ("tile span", pacc[:, 4] - pacc[:, 0])]:
    print(f"  {nm:12s} mean {d.mean() / 100:7.2f} us  max {d.max() / 100:7.2f} us")
pst = pacc[:, 0] / 100
xcc = phw[:, 1] & 0xF
print("  tile start by XCC (mean / max us): " + "  ".join(f"{x}: {pst[xcc == x].mean():.2f}/{pst[xcc == x].max():.2f}" for x in range(8) if (xcc == x).any()))
print("  tile start by tile index eighth (mean us): " + " ".join(f"{pst[k * T // 8:(k + 1) * T // 8].mean():.2f}" for k in range(8)))
print("  tile end by XCC (mean / max us): " + "  ".join(f"{x}: {pacc[xcc == x, 4].mean() / 100:.2f}/{pacc[xcc == x, 4].max() / 100:.2f}" for x in range(8) if (xcc == x).any()))
print(f"sum workgroups (previous round) start {sacc[:, 0].min() / 100:.2f}..{sacc[:, 0].max() / 100:.2f} us, last end {sacc[:, 2].max() / 100:.2f} us")
for nm, d in [("atomics", sacc[:, 1] - sacc[:, 0]), ("responses", sacc[:, 2] - sacc[:, 1])]:
    print(f"  {nm:12s} mean {d.mean() / 100:7.2f} us  max {d.max() / 100:7.2f} us")
print(f"bucket pass starts {acc[:, 0].min() / 100:.2f} us after the partition launch started")
print(f"N={N} buckets={NB} passes={acc[:, 8].mean():.2f}: start spread {acc[:, 0].min() / 100:.2f}..{acc[:, 0].max() / 100:.2f} us")
for nm, d in [("prologue", acc[:, 1] - acc[:, 0]), ("count scan", acc[:, 2] - acc[:, 1]), ("map+issue", acc[:, 3]),
              ("gather wait", acc[:, 4]), ("rank+place", acc[:, 5]), ("V stores", acc[:, 6])]:
    print(f"  {nm:12s} mean {d.mean() / 100:7.2f} us  max {d.max() / 100:7.2f} us")
print(f"  last bucket end {acc[:, 7].max() / 100:.2f} us; mean span {(acc[:, 7] - acc[:, 0]).mean() / 100:.2f} us")
span = (acc[:, 7] - acc[:, 0]) / 100
o = np.argsort(span)
print("span percentiles (us): " + " ".join(f"p{q}={np.percentile(span, q):.1f}" for q in (0, 10, 50, 90, 100)))
print("mean span by blockIdx % 8: " + " ".join(f"{span[x::8].mean():.1f}" for x in range(8)))
print("mean span by blockIdx // 64: " + " ".join(f"{span[k * 64:(k + 1) * 64].mean():.1f}" for k in range(NB // 64)))
print("slowest 16 blocks:", o[-16:].tolist())
print("block start of the slowest vs fastest (us):", f"{acc[o[-16:], 0].mean() / 100:.2f}", f"{acc[o[:16], 0].mean() / 100:.2f}")
cu = (hw[:, 0] >> 8) & 0xF
sh = (hw[:, 0] >> 12) & 1
se = (hw[:, 0] >> 13) & 7
xcc = hw[:, 1] & 0xF
place = xcc * 1000 + se * 100 + sh * 16 + cu
ids, cnts = np.unique(place, return_counts=True)
print("distinct CUs used:", len(ids), " blocks per CU histogram:", dict(zip(*np.unique(cnts, return_counts=True))))
print("touches per bucket: min", hw[:, 2].min(), "max", hw[:, 2].max())
for b in o[-8:]:
    mates = [int(x) for x in np.nonzero(place == place[b])[0] if x != b]
    print(f"  slow block {b}: xcc {xcc[b]} se {se[b]} sh {sh[b]} cu {cu[b]} span {span[b]:.1f} us; CU mates {mates} spans {[round(span[m], 1) for m in mates]}")
