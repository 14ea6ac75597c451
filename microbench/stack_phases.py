"""Phase timings of st_tile_kernel (diagnostic; run on the GPU box).

Opens a stack replica with NRG_EXP=2 (timestamps), replays rounds of N ops over a
50,000-element stack and prints, per phase, the mean and max over tiles of the time since the
tile's start (wall_clock64, 100 MHz), plus the spread of tile start times.
Usage: NRG_EXP=2 python microbench/stack_phases.py [N]
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
dev = nrgpu.DeviceReplica(L.NRG_DS_STACK, 0, max_batch=N, stack_capacity=N * 4 + 100_000,
                          log_bytes=64 * 4 * max(N, 8192))
dev.use_torch_stream()
dev.st_init(list(range(50_000)))
ops = torch.empty(N, dtype=torch.int64, device="cuda")
dev.gen_stack_ops_device(ops, N, 12345)
resp = torch.empty(N, dtype=torch.int32, device="cuda")
some = torch.empty(N, dtype=torch.uint8, device="cuda")
tiles = (N + 8191) // 8192
names = ["loads", "local pass", "scan+responses", "lookback", "query list+sparse table", "queries", "table"]
acc = np.zeros((tiles, 8))
R = 20
for r in range(R + 3):
    dev.st_round_device(ops, N, 1, resp, some)
    torch.cuda.synchronize()
    buf = np.zeros(tiles * 16, np.uint64)
    L.check(L.load().nrg_test_debug_read(dev.handle, buf.ctypes.data_as(C.c_void_p), tiles * 16))
    t = buf.reshape(tiles, 16)[:, :8].astype(np.float64)
    if r >= 3:
        acc += t - t[:, :1].min()
acc /= R
start = acc[:, 0]
print(f"N={N} tiles={tiles}: tile start spread {start.min() / 100:.2f}..{start.max() / 100:.2f} us")
for k, nm in enumerate(names):
    d = (acc[:, k + 1] - acc[:, k]) / 100.0
    print(f"  {nm:14s} mean {d.mean():7.2f} us  max {d.max():7.2f} us")
end = acc[:, 7] / 100.0
print(f"  last tile end {end.max():.2f} us after the first start; mean tile span {(acc[:, 7] - acc[:, 0]).mean() / 100:.2f} us")
