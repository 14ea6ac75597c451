"""Diagnostic (a build with extra marks in st_tile_role's build(): slots 9, 10, 8 by wave 0, 14 by wave 1):
where the time between a tile's aggregate publication and its query structures goes. Run on the GPU box with
NRGPU_LIB pointing at that build. Means over tiles of back-to-back rounds, us from the publication (slot 15)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "node-replication_amd"))
import nrgpu  # noqa: E402
from nrgpu import _lib as L  # noqa: E402

N = 1_000_000
dev = nrgpu.DeviceReplica(L.NRG_DS_STACK, 0, knobs={"EXP": 2}, max_batch=N, stack_capacity=N * 4 + 100_000,
                          pipeline=1, log_bytes=64 * 4 * N)
dev.use_torch_stream()
dev.st_init(list(range(50_000)))
BB = 8
opsl = [torch.empty(N, dtype=torch.int64, device="cuda") for _ in range(BB)]
for i, o in enumerate(opsl):
    dev.gen_stack_ops_device(o, N, 12345 + i)
resps = [torch.empty(N, dtype=torch.int32, device="cuda") for _ in range(2)]
somes = [torch.empty(N, dtype=torch.uint8, device="cuda") for _ in range(2)]
tiles = (N + 2047) // 2048
acc = []
for r in range(12):
    for i in range(BB):
        dev.st_round_device(opsl[i], N, 1, resps[i & 1], somes[i & 1])
    torch.cuda.synchronize()
    buf = np.zeros(tiles * 16, np.uint64)
    L.check(L.load().nrg_test_debug_read(dev.handle, buf.ctypes.data_as(C.c_void_p), tiles * 16))
    x = buf.reshape(tiles, 16).astype(np.float64)
    if r >= 2:
        pub = x[:, 15]
        acc.append([(x[:, k] - pub).mean() / 100.0 for k in (9, 10, 8, 14, 12)] +
                   [(np.maximum(x[:, 8], x[:, 14]) - pub).mean() / 100.0])
a = np.mean(acc, 0)
print("us after publication: wave 0 stores issued %.2f; wave 0 query lists written %.2f; wave 0 at the barrier %.2f;"
      " wave 1 at the barrier %.2f; query structures built %.2f; later of waves 0/1 at the barrier %.2f" % tuple(a))
