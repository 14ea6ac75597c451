"""Worker for the multi-process NR round tests (tests/test_parallel.py).

Launched once per rank with RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the environment.
Each rank plays one replica (one NUMA node / one GPU in the reference's terms): per round it
contributes a write segment of its own length, ReplicatedHashMap all-gathers the segments
(gloo here) and every replica replays the identical global log W_0 || W_1 || ..., then
answers its own reads. Every rank checks its responses against a sequential oracle replay of
the same global log (computed locally from the seeds of all ranks), and the final replica
digests are compared across ranks.

--backend cpu : the replica is an oracle-backed test double (host logic only, runs anywhere)
--backend gpu : the replica is nrgpu.DeviceReplica on cuda:0 (every rank shares the one GPU
                of the box; the exchange still goes through gloo)
--mode partitioned : cnr-style key partitions instead (nrgpu.parallel.PartitionedHashMap): rank
                p holds only the keys it owns, Puts and Gets travel to their owners
                (all_to_all_single), answers come back. Every answer must still equal the NR
                replay of the global log, and the partitions' digests must add up to its digest.
"""
import argparse
import datetime
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "node-replication_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle  # noqa: E402


class OracleReplica:
    """Test double with DeviceReplica's round interface, replaying with the CPU oracle."""

    def __init__(self, prefill):
        self.m = oracle.HashMap()
        self.m.prefill_range(prefill, 1)
        self.logs = []

    def hm_round_segments_device(self, gathered, stride, lens, origins, resp_seg, get_keys, R, get_vals,
                                 get_found, prev=None, prev_found=None):
        g = gathered.cpu().numpy().view(np.uint64).reshape(-1, 2)
        for s, n in enumerate(lens):
            seg = g[s * stride:s * stride + n]
            self.logs.append(seg.copy())
            p, pf = self.m.replay(seg[:, 0].copy(), seg[:, 1].copy())
            if s == resp_seg and prev is not None:
                prev[:n].copy_(torch.from_numpy(p.view(np.int64)))
                prev_found[:n].copy_(torch.from_numpy(pf.astype(np.uint8)))
        v, f = self.m.get_batch(get_keys[:R].cpu().numpy().view(np.uint64))
        get_vals[:R].copy_(torch.from_numpy(v.view(np.int64)))
        get_found[:R].copy_(torch.from_numpy(f.astype(np.uint8)))

    def hm_digest(self):
        return tuple(self.m.digest())


class OraclePartition:
    """Test double for one key partition: partitioned_replay() as DeviceReplica's, on the oracle."""

    def __init__(self, prefill, part, parts):
        from nrgpu.parallel import key_owner

        self.m = oracle.HashMap()
        k = np.arange(prefill, dtype=np.uint64)
        k = k[key_owner(k, parts) == part]
        self.m.replay(k, k + np.uint64(1))  # NrHashMap::default restricted to the partition

    def partitioned_replay(self, puts, keys, want_prev):
        p = puts.reshape(-1, 2).numpy().view(np.uint64)
        pv, pf = self.m.replay(p[:, 0].copy(), p[:, 1].copy())
        v, f = self.m.get_batch(keys.numpy().view(np.uint64).copy())
        return (torch.from_numpy(v.view(np.int64).copy()), torch.from_numpy(f.astype(np.uint8)),
                torch.from_numpy(pv.view(np.int64).copy()) if want_prev else None,
                torch.from_numpy(pf.astype(np.uint8)) if want_prev else None)

    def hm_digest(self):
        return tuple(self.m.digest())


def segment(rank, rnd, span):
    W = 300 + 137 * rank + 61 * rnd  # ragged: ranks contribute different lengths each round
    if rnd == 1 and rank == 0:
        W = 0  # an empty segment
    k = oracle.gen_uniform(W, 1000 * rank + 10 * rnd + 1, span)
    v = oracle.gen_raw(W, 1000 * rank + 10 * rnd + 2)
    return k, v


def reads(rank, rnd, span):
    return oracle.gen_uniform(500 + 50 * rank, 1000 * rank + 10 * rnd + 3, span)


def phase(msg):
    """Progress on stderr, so a stalled rank shows where it stopped (tests/test_parallel.py)."""
    print(f"[dist_worker {os.environ.get('RANK')}] {msg}", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", choices=["cpu", "gpu"], default="cpu")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--span", type=int, default=3000)
    ap.add_argument("--prefill", type=int, default=1000)
    ap.add_argument("--mode", choices=["replicated", "partitioned"], default="replicated")
    a = ap.parse_args()
    phase("init_process_group")
    dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=90))
    rank, world = dist.get_rank(), dist.get_world_size()
    phase(f"rank {rank}/{world} joined")
    from nrgpu.parallel import ReplicatedHashMap

    if a.mode == "partitioned":
        return partitioned(a, rank, world)
    if a.backend == "gpu":
        import nrgpu

        dev_t = torch.device("cuda", 0)
        torch.cuda.set_device(0)
        rep = nrgpu.DeviceReplica(nrgpu._lib.NRG_DS_HASHMAP, 0, log2_slots=16, max_batch=1 << 14,
                                  replica_id=rank + 1)
        rep.hm_prefill_range(a.prefill, 1)
    else:
        dev_t = torch.device("cpu")
        rep = OracleReplica(a.prefill)
    phase("replica ready")
    group = ReplicatedHashMap(rep, device=dev_t)

    model = oracle.HashMap()  # sequential replay of the global log, as one nr thread would see it
    model.prefill_range(a.prefill, 1)
    ok = True
    for rnd in range(a.rounds):
        phase(f"round {rnd}")
        k, v = segment(rank, rnd, a.span)
        W = len(k)
        puts = torch.from_numpy(np.stack([k, v], 1).view(np.int64).copy()).to(dev_t)
        gk = torch.from_numpy(reads(rank, rnd, a.span).view(np.int64).copy()).to(dev_t)
        R = gk.shape[0]
        gv = torch.zeros(R, dtype=torch.int64, device=dev_t)
        gf = torch.zeros(R, dtype=torch.uint8, device=dev_t)
        pv = torch.zeros(max(W, 1), dtype=torch.int64, device=dev_t)
        pf = torch.zeros(max(W, 1), dtype=torch.uint8, device=dev_t)
        group.round(puts.reshape(W, 2), gk, gv, gf, pv, pf)
        if a.backend == "gpu":
            rep.sync()
        # expected: every rank's segment in rank order, then this rank's reads
        for r in range(world):
            kr, vr = segment(r, rnd, a.span)
            p, f = model.replay(kr, vr)
            if r == rank and W:
                ok &= np.array_equal(pv[:W].cpu().numpy().view(np.uint64), p)
                ok &= np.array_equal(pf[:W].cpu().numpy(), f.astype(np.uint8))
        ev, ef = model.get_batch(reads(rank, rnd, a.span))
        ok &= np.array_equal(gv.cpu().numpy().view(np.uint64), ev)
        ok &= np.array_equal(gf.cpu().numpy(), ef.astype(np.uint8))
    dig = [int(x) for x in rep.hm_digest()]
    ok &= dig == [int(x) for x in model.digest()]
    digs = [None] * world
    dist.all_gather_object(digs, dig)
    ok &= all(d == digs[0] for d in digs)  # replicas_are_equal (nr/tests/stack.rs:434-489)
    print(json.dumps({"rank": rank, "ok": bool(ok), "digest": dig}), flush=True)
    dist.destroy_process_group()
    if a.backend == "gpu":
        rep.close()
    sys.exit(0 if ok else 1)


def partitioned(a, rank, world):
    from nrgpu.parallel import PartitionedHashMap

    if a.backend == "gpu":
        import nrgpu

        dev_t = torch.device("cuda", 0)
        torch.cuda.set_device(0)
        rep = nrgpu.DeviceReplica(nrgpu._lib.NRG_DS_HASHMAP, 0, log2_slots=16, max_batch=1 << 14,
                                  replica_id=rank + 1)
        rep.hm_prefill_partition(a.prefill, 1, rank, world)
    else:
        dev_t = torch.device("cpu")
        rep = OraclePartition(a.prefill, rank, world)
    pm = PartitionedHashMap(rep)
    model = oracle.HashMap()  # the NR replay of the global log
    model.prefill_range(a.prefill, 1)
    ok = True
    for rnd in range(a.rounds):
        phase(f"round {rnd}")
        k, v = segment(rank, rnd, a.span)
        W = len(k)
        puts = torch.from_numpy(np.stack([k, v], 1).view(np.int64).copy()).reshape(W, 2).to(dev_t)
        gk = torch.from_numpy(reads(rank, rnd, a.span).view(np.int64).copy()).to(dev_t)
        R = gk.shape[0]
        gv = torch.full((R,), -1, dtype=torch.int64, device=dev_t)
        gf = torch.full((R,), 7, dtype=torch.uint8, device=dev_t)
        want = rnd != 1 or rank != 1  # a rank without previous values in round 1
        pv = torch.full((W,), -1, dtype=torch.int64, device=dev_t) if want else None
        pf = torch.full((W,), 7, dtype=torch.uint8, device=dev_t) if want else None
        pm.round(puts, gk, gv, gf, pv, pf)
        for r in range(world):
            kr, vr = segment(r, rnd, a.span)
            p, f = model.replay(kr, vr)
            if r == rank and want:
                ok &= np.array_equal(pv.cpu().numpy().view(np.uint64), p)
                ok &= np.array_equal(pf.cpu().numpy(), f.astype(np.uint8))
        ev, ef = model.get_batch(reads(rank, rnd, a.span))
        ok &= np.array_equal(gv.cpu().numpy().view(np.uint64), ev)
        ok &= np.array_equal(gf.cpu().numpy(), ef.astype(np.uint8))
    dig = [int(x) for x in rep.hm_digest()]
    digs = [None] * world
    dist.all_gather_object(digs, dig)
    total = [sum(d[0] for d in digs), sum(d[1] for d in digs) % (1 << 64), 0]
    for d in digs:
        total[2] ^= d[2]
    ok &= total == [int(x) for x in model.digest()]  # the partitions add up to the NR replica
    print(json.dumps({"rank": rank, "ok": bool(ok), "digest": total}), flush=True)
    dist.destroy_process_group()
    if a.backend == "gpu":
        rep.close()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
