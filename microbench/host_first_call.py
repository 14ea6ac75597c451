"""Host time of the first nrg_hashmap_round_async call after a device sync, under variants of
what runs between the previous rounds and the sync (diagnostic for the 20-step bench line,
whose first call takes ~20 us against ~5 us for the rest).
Usage: python microbench/host_first_call.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "node-replication_amd")]

import torch  # noqa: E402

import nrgpu  # noqa: E402
from nrgpu import _lib as L  # noqa: E402

W, R, P = 100_000, 900_000, 8
rep = nrgpu.DeviceReplica(L.NRG_DS_HASHMAP, 0, log2_slots=26, max_batch=W, log_bytes=64 * 4 * W, pipeline=1)
stream = torch.cuda.Stream()
torch.cuda.set_stream(stream)
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


def call(i):
    fn(h, ptrs[i % P][0], W, 1, ptrs[i % P][1], R, gv.data_ptr(), gf.data_ptr(), None, None)


def region(before, label, reps=6):
    out = []
    for _ in range(reps):
        for i in range(5):
            call(i)
        rep.sync()
        before()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        call(0)
        t1 = time.perf_counter()
        call(1)
        t2 = time.perf_counter()
        rep.join()
        torch.cuda.synchronize()
        out.append((round((t1 - t0) * 1e6, 1), round((t2 - t1) * 1e6, 1)))
    print(f"{label:40s} first two calls (us): {out}", flush=True)


def nothing():
    pass


def sleep_1ms():
    time.sleep(0.001)


def spin_1ms():
    t = time.perf_counter()
    while time.perf_counter() - t < 0.001:
        pass


def torch_work():
    torch.unique(gk[0, :100000])


def stderr_print():
    print("x", file=sys.stderr, flush=True)


for f, lab in [(nothing, "nothing"), (sleep_1ms, "sleep 1 ms"), (spin_1ms, "spin 1 ms"), (torch_work, "torch.unique (syncs)"),
               (stderr_print, "print to stderr"), (nothing, "nothing again")]:
    region(f, lab)
