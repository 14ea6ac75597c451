"""Host time of each nrg_hashmap_round_async call right after a device sync (diagnostic).

The driver's 20-step bench line pays a fixed cost per timed region; the kernel trace shows the
GPU idle for ~26 us after the first launch because the second call takes that long on the host.
This replays B1 rounds after a sync and prints the host microseconds of the first calls, for
the pipelined rounds the bench uses and, for comparison, with the deferred half flushed at once.
Usage: python microbench/host_steps.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "node-replication_amd")]

import torch  # noqa: E402

import nrgpu  # noqa: E402
from nrgpu import _lib as L  # noqa: E402


def run(pipeline, label):
    W, R, P = 100_000, 900_000, 8
    rep = nrgpu.DeviceReplica(L.NRG_DS_HASHMAP, 0, log2_slots=26, max_batch=W, log_bytes=64 * 4 * W,
                              pipeline=pipeline)
    rep.use_torch_stream()
    rep.hm_prefill_range(1 << 23, 1)
    puts = torch.empty((P, W, 2), dtype=torch.int64, device="cuda")
    gk = torch.empty((P, R), dtype=torch.int64, device="cuda")
    tk = torch.empty(W, dtype=torch.int64, device="cuda")
    tv = torch.empty(W, dtype=torch.int64, device="cuda")
    for p in range(P):
        rep.gen_uniform_device(tk, W, 100 + p, 10_000_000)
        rep.gen_raw_device(tv, W, 200 + p)
        rep.gen_puts_device(puts[p], tk, tv, W)
        rep.gen_uniform_device(gk[p], R, 300 + p, 10_000_000)
    gv = torch.empty(R, dtype=torch.int64, device="cuda")
    gf = torch.empty(R, dtype=torch.uint8, device="cuda")
    fn, h = rep._lib.nrg_hashmap_round_async, rep._h
    ptrs = [(puts[p].data_ptr(), gk[p].data_ptr()) for p in range(P)]
    for rnd in range(4):
        for i in range(5):
            fn(h, ptrs[i % P][0], W, 1, ptrs[i % P][1], R, gv.data_ptr(), gf.data_ptr(), None, None)
        rep.sync()
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        for i in range(6):
            fn(h, ptrs[i % P][0], W, 1, ptrs[i % P][1], R, gv.data_ptr(), gf.data_ptr(), None, None)
            t.append(time.perf_counter())
        rep.join()
        t.append(time.perf_counter())
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        d = [round((b - a) * 1e6, 1) for a, b in zip(t, t[1:])]
        print(f"{label} region {rnd}: host us per call {d[:6]} join {d[6]} sync {d[7]}", flush=True)
    rep.close()


if __name__ == "__main__":
    run(1, "pipeline=1")
    run(0, "pipeline=0")
