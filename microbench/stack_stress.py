"""Stack race stress: bench-size rounds (1M ops, 50/50) plain and pipelined, every Pop answer
compared with the sequential oracle; prints TOTAL_BAD. NRGPU_LIB picks the build, ROUNDS the count."""
import os, sys, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "node-replication_amd"), os.path.join(ROOT, "oracle")]
import nrgpu, oracle as orc
n = 1_000_000
R = int(os.environ.get("ROUNDS", "24"))
tot_bad = 0
for pipe in (0, 1):
    dev = nrgpu.DeviceReplica(nrgpu._lib.NRG_DS_STACK, 0, max_batch=n, stack_capacity=1 << 22, log_bytes=64 * 4 * n, pipeline=pipe)
    init = np.arange(50_000, dtype=np.uint32)
    dev.st_init(init)
    os_ = orc.Stack(init)
    outs = []
    for r in range(R):
        vals, ops = orc.gen_stack_ops(n, 0x5AC + r + 100 * pipe)
        rec = np.zeros(n, nrgpu.STACK_OP_DTYPE); rec["val"] = vals; rec["op"] = ops
        d_ops = torch.from_numpy(rec.view(np.int64).copy()).cuda()
        resp = torch.zeros(n, dtype=torch.int32, device="cuda")
        some = torch.zeros(n, dtype=torch.uint8, device="cuda")
        dev.st_round_device(d_ops, n, 1, resp, some)
        outs.append((resp, some, os_.replay(vals, ops), ops))
        if len(outs) >= 4 or r == R - 1:
            dev.join() if pipe else None
            torch.cuda.synchronize()
            for resp, some, (oresp, osome), ops in outs:
                a = resp.cpu().numpy().view(np.uint32); s = some.cpu().numpy()
                bad = np.nonzero((a != oresp) | (s != osome))[0]
                tot_bad += len(bad)
                for i in bad[:4]:
                    print("  pipe", pipe, "i", i, "op", ops[i], "got", a[i], s[i], "want", oresp[i], osome[i], flush=True)
            outs = []
    print("pipeline", pipe, "rounds", R, "bad so far", tot_bad, flush=True)
print("TOTAL_BAD", tot_bad)
