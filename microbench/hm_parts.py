"""Time the pieces of the B1 NrHashMap round separately (HIP events around each kernel):
gets only, puts only (K1 + apply), and the fused round. Used to decide where a round's time
goes before tuning; not part of the product."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "node-replication_amd")]

import torch  # noqa: E402

import nrgpu  # noqa: E402
from nrgpu import _lib as L  # noqa: E402


def main():
    W, R, steps = 100_000, 900_000, 200
    rep = nrgpu.DeviceReplica(L.NRG_DS_HASHMAP, 0, log2_slots=26, max_batch=W, log_bytes=64 * 4 * W,
                              pipeline=int(os.environ.get("PIPE", "0")))
    rep.use_torch_stream()
    rep.hm_prefill_range(1 << 23, 1)
    P = 32
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
    torch.cuda.synchronize()

    last = {}

    def run(name, fn):
        for i in range(10):
            fn(i)
        torch.cuda.synchronize()
        rep.kernel_timing(True)
        t = time.perf_counter()
        for i in range(steps):
            fn(i)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t) / steps * 1e6
        parts = {}
        for k in ("hm_index", "hm_apply", "hm_get"):
            n, ms = rep.kernel_time(k)  # cumulative: report the delta of this run
            n0, ms0 = last.get(k, (0, 0.0))
            last[k] = (n, ms)
            parts[k] = round((ms - ms0) * 1e3 / (n - n0), 2) if n > n0 else None
        rep.kernel_timing(False)
        print(f"{name:28s} {el:8.2f} us/step  kernels(avg us): {parts}", flush=True)

    run("gets only (900k)", lambda i: rep.hm_get_device(gk[i % P], R, gv, gf))
    run("puts only (100k)", lambda i: rep.hm_round_device(puts[i % P], W, 1, None, 0, None, None))
    run("round 100k put + 900k get", lambda i: rep.hm_round_device(puts[i % P], W, 1, gk[i % P], R, gv, gf))
    # host floor: tiny rounds (1 put, 1 get) are launch/host bound
    run("host floor (1 put + 1 get)", lambda i: rep.hm_round_device(puts[i % P], 1, 1, gk[i % P], 1, gv, gf))
    # raw ctypes call with precomputed pointers (no torch indexing / python wrapper)
    import ctypes as C

    f = rep._lib.nrg_hashmap_round_async
    h = rep.handle
    pp = [C.c_void_p(puts[p].data_ptr()) for p in range(P)]
    gp = [C.c_void_p(gk[p].data_ptr()) for p in range(P)]
    gvp, gfp = C.c_void_p(gv.data_ptr()), C.c_void_p(gf.data_ptr())
    run("round via raw ctypes", lambda i: f(h, pp[i % P], W, 1, gp[i % P], R, gvp, gfp, None, None))


if __name__ == "__main__":
    main()
