#!/usr/bin/env python3
"""bench.py — NR log-replay throughput on MI355X (BASELINE.json metric).

Metric: whole-node Mops/s of an NrHashMap replica group at 10% writes (BASELINE.json
"Mops/s whole node, NrHashMap 10% writes, 1/2/4/8 GPUs; replay HBM GB/s vs peak").

Workload (N = 1: BASELINE.json configs[1], "B1" in SURVEY.md §8d): one GPU replica with a
2^26-slot open-addressing u64->u64 table (1 GiB), prefilled with keys [0, 2^23) -> k+1
(NrHashMap::default, benches/hashmap.rs:91-100), uniform keys over a 10M key space, rounds
of 1M ops = 100k Put + 900k Get per GPU. One step = one NR round on every GPU:
  Log::append of the rank's write segment (RCCL all-gather of all ranks' segments for N > 1)
  -> Log::exec of the round's global writes -> dispatch of the rank's reads after sync
  (nr/src/replica.rs:544-595, :483-497), fused into nrg_hashmap_round[_segments]_async.
Put responses follow benches/hashmap.rs:114-119 (Ok(None)); the variant with HashMap::insert's
previous-value responses (nr/examples/hashmap.rs:46-50) is measured beside it.
Inputs are generated on device before the timed region (a pool of distinct batches, cycled).
For N > 1 every rank adds 1M ops per round (weak scaling); the value counts all ranks' ops.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "node-replication_amd"), os.path.join(ROOT, "oracle")]

METRIC = "Mops/s whole node, NrHashMap 10% writes, 1/2/4/8 GPUs; replay HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


class Watchdog:
    """Whole-process deadline. A rank stuck in a collective -- a peer that never joined, an RCCL
    round that never completes, a blocked ncclCommInitRank -- ends the run non-zero with a
    diagnostic naming the rank and the phase instead of holding the driver's slot. (The replica
    group's own deadline, nrg_group_set_timeout / --group-timeout-ms, turns a missing peer inside a
    round into NRG_E_TIMEOUT first; this covers what that cannot reach.)"""

    def __init__(self):
        self.phase = "start"
        self.rank = int(os.environ.get("RANK", "0"))

    def arm(self, seconds: float):
        if seconds > 0:
            threading.Thread(target=self._fire, args=(seconds,), daemon=True).start()

    def _fire(self, seconds):
        time.sleep(seconds)
        log(f"watchdog: rank {self.rank} of {os.environ.get('WORLD_SIZE', '1')} still in phase '{self.phase}' "
            f"after {seconds:.0f} s (a peer rank stalled or never joined?); exiting with status 3")
        os._exit(3)


WATCH = Watchdog()


def numa_groups(cpus):
    """Group the CPUs we may run on by NUMA node (/sys/devices/system/node)."""
    groups = {}
    base = "/sys/devices/system/node"
    node_of = {}
    try:
        for d in os.listdir(base):
            if not d.startswith("node") or not d[4:].isdigit():
                continue
            with open(os.path.join(base, d, "cpulist")) as f:
                for part in f.read().strip().split(","):
                    if not part:
                        continue
                    a, _, b = part.partition("-")
                    for c in range(int(a), int(b or a) + 1):
                        node_of[c] = int(d[4:])
    except OSError:
        pass
    for c in cpus:
        groups.setdefault(node_of.get(c, 0), []).append(c)
    return [groups[k] for k in sorted(groups)]


def cpu_budget(n_affinity: int) -> int:
    """CPUs this job may really use: the affinity mask, capped by the cgroup CPU quota and by
    OMP_NUM_THREADS (the GPU box gives one GPU's job a 16-CPU share of a larger host)."""
    n = n_affinity
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
            if q != "max":
                n = min(n, max(1, int(int(q) / int(p))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        n = min(n, int(omp))
    return max(1, n)


def host_topology():
    """nproc, physical cores, SMT state and NUMA node count of this host (BASELINE.md §2;
    the reference's harness records its topology the same way, benches/mkbench.rs:592-604)."""
    cores = set()
    base = "/sys/devices/system/cpu"
    try:
        for d in os.listdir(base):
            if d.startswith("cpu") and d[3:].isdigit():
                try:
                    with open(os.path.join(base, d, "topology", "core_id")) as f:
                        core = f.read().strip()
                    with open(os.path.join(base, d, "topology", "physical_package_id")) as f:
                        pkg = f.read().strip()
                    cores.add((pkg, core))
                except OSError:
                    pass
    except OSError:
        pass
    smt = None
    try:
        with open(os.path.join(base, "smt", "active")) as f:
            smt = f.read().strip() == "1"
    except OSError:
        pass
    try:
        numa = len([d for d in os.listdir("/sys/devices/system/node") if d.startswith("node") and d[4:].isdigit()])
    except OSError:
        numa = None
    return {"nproc": os.cpu_count(), "physical_cores": len(cores) or None, "smt": smt, "numa_nodes": numa,
            "cpus_allowed": len(os.sched_getaffinity(0)), "cpu_budget": cpu_budget(len(os.sched_getaffinity(0)))}


def _nr_cpu_run(seconds, write_ratio, key_space, prefill, threads=None):
    """One run of the C++ restatement of nr (flat combining + shared log + per-replica RwLock),
    one Replica per NUMA node over the threads used (oracle/nr_cpu.cpp)."""
    import oracle

    # the thread budget spread evenly over the NUMA nodes (lowest-numbered CPUs of each node are
    # physical cores; their SMT siblings come later), one Replica per node
    cpu_list, rep, groups = _nr_groups(threads)
    res = oracle.nr_hashmap_bench(cpu_list, rep, seconds, write_ratio, key_space, prefill, 2_500_000, 0xC0FFEE)
    return res, cpu_list, groups


def cpu_baseline(seconds: float, write_ratio: int, key_space: int, prefill: int):
    """The B1 stream through the C++ restatement of nr on this host's cores (the reported
    baseline), plus BASELINE configs[0] as the reference defines it (5M keys, prefill 2^22,
    5 s, benches/hashmap.rs:30-48) and a 1-thread point."""
    res, cpu_list, groups = _nr_cpu_run(seconds, write_ratio, key_space, prefill)
    out = {
        "value": round(res.ops / res.seconds / 1e6, 3),
        "unit": "Mops/s",
        "cores": len(cpu_list),
        "kind": "port",
        "sample": (f"{res.seconds:.1f} s of the same NrHashMap stream (uniform over {key_space} keys, prefill "
                   f"[0,{prefill}), {write_ratio}% writes, 2.5M-op per-thread shuffles, 128 ops per clock check) "
                   f"through the C++ restatement of nr on {len(cpu_list)} threads, {len(groups)} replica(s) "
                   f"(one per NUMA node); {res.ops} ops"),
        "host": host_topology(),
    }
    side = min(5.0, seconds)  # the configs[0] and 1-thread legs
    c0, c0_cpus, c0_groups = _nr_cpu_run(side, 10, 5_000_000, 1 << 22)
    out["configs0"] = {"value": round(c0.ops / c0.seconds / 1e6, 3), "unit": "Mops/s", "cores": len(c0_cpus),
                       "replicas": len(c0_groups),
                       "sample": f"BASELINE configs[0]: 5M keys, prefill [0,2^22), uniform, 10% writes, "
                                 f"{c0.seconds:.1f} s"}
    t1, _, _ = _nr_cpu_run(side, write_ratio, key_space, prefill, threads=1)
    out["one_thread"] = {"value": round(t1.ops / t1.seconds / 1e6, 3), "unit": "Mops/s", "cores": 1,
                         "sample": "the B1 stream on 1 thread, 1 replica, %.1f s" % t1.seconds}
    return out


def traffic_key(args):
    if args.workload == "stack":
        return "stack_ops%d_init%d_n%d" % (args.ops_per_gpu, args.stack_init, int(os.environ.get("WORLD_SIZE", "1")))
    if args.workload == "synthetic":
        return "synthetic_ops%d_n%d" % (args.ops_per_gpu, int(os.environ.get("WORLD_SIZE", "1")))
    return "w%d_ops%d_ks%d_pf%d_s%d_%s_n%d%s" % (args.write_ratio, args.ops_per_gpu, args.key_space, args.prefill,
                                                args.log2_slots, key_dist_name(args),
                                                int(os.environ.get("WORLD_SIZE", "1")),
                                                "_part" if getattr(args, "partitioned", False) else "")


def key_dist_name(args):
    if args.dist == "uniform":
        return "uniform"
    return "zipf%g%s" % (args.theta, "s" if args.scramble else "")


def measured_traffic(args):
    """HBM bytes per launch of the dominant kernel from the PMC passes of tools/profile.sh
    (FETCH_SIZE x2 + WRITE_SIZE, gfx950 correction per MI355X_MICROARCH.md), as committed by
    tools/prof_summary.py for this exact workload; None when no matching profile exists."""
    path = os.path.join(ROOT, "profiles", "traffic_hm_round.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    e = t.get(traffic_key(args))
    if not e:
        return None
    return {"bytes_per_launch": e["bytes_per_launch"], "source": e["source"]}


class Env:
    """Process/distributed context of one bench run (one process per GPU)."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        local = int(os.environ.get("LOCAL_RANK", "0"))
        # main() refuses a WORLD_SIZE that disagrees with --gpus before any GPU call
        assert self.world == args.gpus, (self.world, args.gpus)
        if args.share_gpu:
            local = 0  # rehearsal of the N > 1 path with every rank on the box's one GPU (gloo only)
        self.local = local
        self.opening = args.opening
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        # one non-blocking stream for the replica and this process's torch work (the null
        # stream would order against every blocking stream, RCCL's included)
        self.stream = torch.cuda.Stream(self.dev)
        torch.cuda.set_stream(self.stream)
        WATCH.phase = "init_process_group"
        if self.world > 1:
            if args.backend == "nccl":
                dist.init_process_group("nccl", device_id=self.dev)  # RCCL over xGMI
            else:
                dist.init_process_group("gloo")

    first_calls = []  # host us of the first step of every timed region of the process (diagnostic)

    def timed(self, n, step, rep, host_s=None, finish=None, evs=None):
        """Barrier + sync, K steps, the replica's deferred work launched, sync + barrier; max over
        ranks of the wall time. evs: {i: torch.cuda.Event} recorded on the stream right after
        step i (the roofline window; the timed region proper passes none)."""
        torch, dist = self.torch, self.dist
        # Python's cyclic GC runs on allocation counts: held off inside the timed region (a
        # collection right before it made the first host call 50+ us: caches walked cold)
        gc.disable()
        try:
            if self.world > 1:
                dist.barrier()
            if self.opening in ("spin", "keep"):
                # wait for the device with the host thread awake (a blocking sync parks it, and the
                # first calls after the wake-up ran 20-80 us slow), then keep the core busy briefly.
                # "keep" (A/B): the device stays busy too, on a ~100-us spin kernel, until just
                # before the region opens
                if self.opening == "keep":
                    torch.cuda._sleep(200_000)
                ev = torch.cuda.Event()
                ev.record()
                while not ev.query():
                    pass
                if self.opening == "spin":
                    t_end = time.perf_counter() + 1e-3
                    while time.perf_counter() < t_end:
                        pass
            torch.cuda.synchronize()
            t = time.perf_counter()
            marks = [t]
            for i in range(n):
                step(i)
                if evs is not None and i in evs:
                    evs[i].record()
                if i < 3:
                    marks.append(time.perf_counter())
            # launches the last round's deferred apply + reads (and completes a pipelined group
            # round): inside the timed region
            if finish is not None:
                finish()
            else:
                rep.join()
            if host_s is not None:
                host_s[0] = time.perf_counter() - t
                host_s[1:] = [round((b - a) * 1e6, 2) for a, b in zip(marks, marks[1:])]
            if len(marks) > 1:
                Env.first_calls.append(round((marks[1] - marks[0]) * 1e6, 1))
            torch.cuda.synchronize()
            if self.world > 1:
                dist.barrier()
            el = time.perf_counter() - t
        finally:
            gc.enable()
        if self.world > 1:
            x = torch.tensor([el], dtype=torch.float64, device=self.dev)
            dist.all_reduce(x, op=dist.ReduceOp.MAX)
            el = float(x.item())
        return el

    def close(self):
        if self.world > 1:
            self.dist.destroy_process_group()


def apply_knobs(rep, args):
    for kv in args.knob:
        name, _, v = kv.partition("=")
        rep.set_knob(name.strip().upper(), int(v, 0))


def common_fields(args, env, value, ms_per_step, metric, dtype, config):
    return {
        "metric": metric,
        "value": round(value, 3),
        "unit": "Mops/s",
        "n_gpus": env.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": dtype,
        "data": "synthetic",
        "config": config,
    }


ROOF_ROUNDS = 64  # rounds of the roofline region (at least --steps)


def roofline_region(args, rep, run, names):
    """Kernel durations for the roofline, measured right after the timed region on the same
    stream and workload (the timed region itself carries no events, so `value` is the
    unperturbed rate), two ways:
    * window (the line's avg_launch_us): a run of n = max(steps, ROOF_ROUNDS) rounds with one
      HIP event on the stream after round 0's call and one after round n-1's; rounds 1..n-1 are
      steady-state launches of the round's kernel(s), one round of work each, and nothing else
      runs on the stream, so (stop - start) / (n - 1) is the per-round kernel time with no event
      on any dispatch. Idle gaps between launches would count in it: it can only overstate.
    * bracketed: another n rounds with every timing_every-th launch of the named kernels carrying
      HIP events stamped from its own dispatch (hipExtLaunchKernelGGL). Those launches run
      longer than unbracketed ones (stack: ~17 % over rocprof's duration,
      profiles/r02_s8_event_bracketing.txt), so this is reported beside the window only.
    Returns ({name: (launches, total_ms)}, (window rounds, window ms))."""
    if args.no_kernel_timing:
        return {n: (0, 0.0) for n in names}, (0, 0.0)
    torch = sys.modules["torch"]
    nwin = max(args.steps, ROOF_ROUNDS)
    evs = {0: torch.cuda.Event(enable_timing=True), nwin - 1: torch.cuda.Event(enable_timing=True)}
    run(nwin, evs=evs)
    win = (nwin - 1, evs[0].elapsed_time(evs[nwin - 1]))
    rep.kernel_timing(True, only=",".join(names), every=args.timing_every)
    run(nwin)
    out = {n: rep.kernel_time(n) for n in names}
    rep.kernel_timing(False)
    return out, win


def roofline(kernel, k_bytes, k_n, k_ms, args, traffic, win=(0, 0.0)):
    """k_n, k_ms: the bracketed launches (per round of work); win: the window (rounds, ms), which
    gives avg_launch_us and `achieved` when measured."""
    b_avg_s = (k_ms / 1e3 / k_n) if k_n else float("nan")
    w_n, w_ms = win
    k_avg_s = (w_ms / 1e3 / w_n) if w_n else b_avg_s
    achieved = k_bytes / k_avg_s / 1e9 if (w_n or k_n) else None
    return {
        "bound": "hbm",
        "kernel": kernel,
        "achieved": round(achieved, 1) if achieved else None,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
        "traffic": traffic.get("bytes_per_launch") if traffic else None,
        "traffic_source": traffic.get("source") if traffic else None,
        "bytes_per_launch": int(k_bytes),
        "region": ("rounds 1..%d of a %d-round run after the timed region, between two HIP events on the "
                   "kernel's stream (no event on any dispatch); bracketed: another %d rounds, every %d-th "
                   "launch with dispatch-stamped events" % (w_n, w_n + 1, w_n + 1, args.timing_every))
        if w_n else "%d rounds after the timed region, every %d-th launch event-bracketed" % (
            max(args.steps, ROOF_ROUNDS), args.timing_every),
        "traffic_key": traffic_key(args),
        "avg_launch_us": round(k_avg_s * 1e6, 3) if (w_n or k_n) else None,
        "launches": w_n if w_n else k_n,
        "bracketed_avg_launch_us": round(b_avg_s * 1e6, 3) if k_n else None,
        "bracketed_launches": k_n,
        "sampled_every": args.timing_every,
    }


# ---------------------------------------------------------------------------------------------
def run_hashmap(args, env):
    torch = env.torch
    import nrgpu
    from nrgpu import _lib as L

    world, rank, dev_t = env.world, env.rank, env.dev
    W = args.ops_per_gpu * args.write_ratio // 100
    R = args.ops_per_gpu - W
    Wg = W * world
    rep = nrgpu.DeviceReplica(L.NRG_DS_HASHMAP, env.local, log2_slots=args.log2_slots, max_batch=max(Wg, 1),
                              log_bytes=64 * 4 * max(Wg, 8192), replica_id=rank + 1, pipeline=args.pipeline)
    apply_knobs(rep, args)
    rep.use_torch_stream()
    if args.partitioned:  # cnr-style: this rank holds only the keys it owns
        rep.hm_prefill_partition(args.prefill, 1, rank, world)
    else:
        rep.hm_prefill_range(args.prefill, 1)

    # ---- inputs: a pool of distinct batches generated on device (seeds per rank/batch) ----
    P = max(1, min(args.pool, args.steps + args.warmup))
    puts = torch.empty((P, max(W, 1), 2), dtype=torch.int64, device=dev_t)
    gkeys = torch.empty((P, max(R, 1)), dtype=torch.int64, device=dev_t)
    tmp_k = torch.empty(max(W, 1), dtype=torch.int64, device=dev_t)
    tmp_v = torch.empty(max(W, 1), dtype=torch.int64, device=dev_t)
    seed0 = 0x4E52475055310001 + rank * 0x1000193

    def keys_into(out, n, seed):
        if args.dist == "uniform":
            rep.gen_uniform_device(out, n, seed, args.key_space)
        else:
            rep.gen_zipf_device(out, n, seed, args.key_space, args.theta, args.scramble)

    for p in range(P):
        if W:
            keys_into(tmp_k, W, seed0 + 3 * p)
            rep.gen_raw_device(tmp_v, W, seed0 + 3 * p + 1)
            rep.gen_puts_device(puts[p], tmp_k, tmp_v, W)
        if R:
            keys_into(gkeys[p], R, seed0 + 3 * p + 2)
    gvals = torch.empty(max(R, 1), dtype=torch.int64, device=dev_t)
    gfound = torch.empty(max(R, 1), dtype=torch.uint8, device=dev_t)
    pvals = torch.empty(max(W, 1), dtype=torch.int64, device=dev_t)
    pfound = torch.empty(max(W, 1), dtype=torch.uint8, device=dev_t)
    torch.cuda.synchronize()

    # distinct keys per batch (for the algorithmic byte count), outside the timed region
    nb = min(P, 8)
    u_r = sum(int(torch.unique(gkeys[p, :R]).numel()) for p in range(nb)) / nb if R else 0
    u_w_local = sum(int(torch.unique(puts[p, :W, 0]).numel()) for p in range(nb)) / nb if W else 0
    if world > 1:  # distinct keys of the whole round's log (all ranks' segments)
        x = torch.tensor([u_w_local], dtype=torch.float64, device=dev_t if args.backend == "nccl" else "cpu")
        env.dist.all_reduce(x)
        u_w = float(x.item())
    else:
        u_w = u_w_local

    group = cgroup = pgroup = None
    if args.partitioned:
        # Puts and Gets routed to their key's owner (RCCL send/recv in libnrgpu.so)
        from nrgpu.parallel import PartitionedGroup

        if args.backend != "nccl":
            raise SystemExit("--partitioned needs --backend nccl (RCCL send/recv)")
        WATCH.phase = "nrg_group_join (partitioned)"
        pgroup = PartitionedGroup(rep, rank, world, timeout_ms=args.group_timeout_ms)
    elif world > 1 and args.backend == "nccl":
        # the C ABI's replica group: RCCL all-gather on a library-owned stream, replay on ours
        from nrgpu.parallel import ReplicaGroup

        WATCH.phase = "nrg_group_join"
        cgroup = ReplicaGroup(rep, rank, world, timeout_ms=args.group_timeout_ms)
        inputs = torch.cuda.Stream(dev_t)  # inputs exist before the timed region: gathers run ahead
        cgroup.set_input_stream(inputs.cuda_stream)
    elif world > 1:
        from nrgpu.parallel import ReplicatedHashMap

        group = ReplicatedHashMap(rep, device=dev_t)

    # raw device pointers per pool entry, resolved once: the per-round host path is then one
    # C-ABI call (Replica::combine's batch hand-off), not tensor indexing + marshalling
    round_fn, h = rep._lib.nrg_hashmap_round_async, rep._h
    ptrs = [(puts[p].data_ptr(), gkeys[p].data_ptr()) for p in range(P)]
    gv_p, gf_p, pv_p, pf_p = gvals.data_ptr(), gfound.data_ptr(), pvals.data_ptr(), pfound.data_ptr()
    gathered = {}
    mode = {"prev": False, "n": 0}
    seg_lens = [W] * world

    def step(i):
        p = i % P
        prev = mode["prev"]
        if pgroup is not None:
            pp, gp = ptrs[p]
            pgroup.round_async(pp, W, gp, R, gv_p, gf_p, pv_p if prev else None, pf_p if prev else None)
        elif cgroup is not None:
            pp, gp = ptrs[p]
            # every rank's segment is W records: seg_lens keeps the round stream ordered (no length
            # exchange); the round header still checks it on every rank
            cgroup.round_async(pp, W, pv_p if prev else None, pf_p if prev else None, gp, R, gv_p, gf_p,
                               seg_lens=seg_lens)
        elif group is None:
            pp, gp = ptrs[p]
            rc = round_fn(h, pp, W, rank + 1, gp, R, gv_p, gf_p, pv_p if prev else None, pf_p if prev else None)
            if rc:
                L.check(rc, "nrg_hashmap_round_async")
        else:
            # the all-gather of round i+1 is in flight while round i replays
            g = gathered.pop(i) if i in gathered else group.gather_async(puts[p, :W], stride=W)
            if i + 1 < mode["n"]:
                gathered[i + 1] = group.gather_async(puts[(i + 1) % P, :W], stride=W)
            group.replay(g, gkeys[p, :R], gvals, gfound, pvals if prev else None, pfound if prev else None)

    def finish():
        if pgroup is not None:
            pgroup.flush()  # the last pipelined round
        rep.join()

    def run(n, prev=False, host_s=None, evs=None):
        mode["prev"], mode["n"] = prev, n
        return env.timed(n, step, rep, host_s, finish=finish, evs=evs)

    mode["n"] = args.warmup
    WATCH.phase = "warmup rounds"
    for i in range(args.warmup):
        step(i)
    if cgroup is not None or pgroup is not None:
        (cgroup or pgroup).sync()  # bounded by the group's deadline
    rep.sync()
    log(f"rank {rank}: warmup {args.warmup} rounds done")

    # timed region: no HIP events. The dominant (and only per-round) kernel, hm_round, is then
    # timed in the roofline region with events stamped from its own dispatch packets
    # (hipExtLaunchKernelGGL start/stop events on the stream it runs on) on every timing_every-th
    # launch (steady-state launches: round e's index plus round e-1's apply and reads, i.e. one
    # round of work each).
    host_s = [0.0]
    WATCH.phase = "timed region"
    elapsed = run(args.steps, host_s=host_s)  # no events in the timed region
    kt, win = roofline_region(args, rep, run, ["hm_round", "hm_papply"])
    (k_n, k_ms), (a_n, a_ms) = kt["hm_round"], kt["hm_papply"]
    if a_n and k_n:  # partition rounds: hm_round (partition + reads) + hm_papply (the table pass)
        k_ms = k_ms + a_ms * k_n / a_n
    rep.sync()
    value = world * args.ops_per_gpu * args.steps / elapsed / 1e6

    prev_value = None
    if not args.no_prev_variant:
        n2 = max(args.steps // 4, 10)
        e2 = run(n2, prev=True)
        prev_value = world * args.ops_per_gpu * n2 / e2 / 1e6
    rep.sync()
    if rank != 0:
        return None

    # ---- roofline of the dominant kernel (hm_round: index of round e + apply/reads of e-1) ----
    # Algorithmic bytes per round: B = 16 R + 16 W_glob + 64 U_r + 128 U_w
    # (8-B key in + 8-B value out per Get, the 16-B records replayed, one 64-B sector per
    # distinct key read, read + write-back per distinct key written; Put responses are
    # Ok(None) here, so no 8 W_own term). Every sampled launch carries one round of work.
    round_bytes = 16 * R + 16 * Wg + 64 * u_r + 128 * u_w
    dist_txt = ("uniform keys over %d" % args.key_space if args.dist == "uniform" else
                "Zipf(theta=%g%s) keys over %d" % (args.theta, ", scrambled" if args.scramble else ", hot keys adjacent",
                                                   args.key_space))
    metric = METRIC if not args.partitioned else (
        "Mops/s whole node, NrHashMap key-partitioned rounds (cnr-style, SURVEY.md 8 f4; not the NR headline)")
    res = common_fields(args, env, value, elapsed * 1e3 / args.steps, metric, "u64", {
        "workload": ("NrHashMap replica per GPU: 2^%d-slot table, %s, prefill [0,%d)->k+1, rounds of %d ops/GPU "
                     "= %d Put + %d Get%s" % (
                         args.log2_slots, dist_txt, args.prefill, args.ops_per_gpu, W, R,
                         "; write segments all-gathered (%s), every replica replays all %d Puts" % (
                             "RCCL over xGMI from libnrgpu.so's replica group" if args.backend == "nccl"
                             else "gloo rehearsal", Wg)
                         if world > 1 and not args.partitioned else "") +
                     ("; key-partitioned: rank p holds the keys with nrg_key_owner(k, %d) == p, Puts and Gets "
                      "routed to their owners and answers back (RCCL send/recv)%s" % (
                          world, "; one rank owns every key: partition and route-back are the identity, the "
                          "replay reads the caller's records and answers into its buffers" if world == 1 else "")
                      if args.partitioned else "")),
        "baseline_config": "configs[1] (B1)" if (world == 1 and args.write_ratio == 10 and args.dist == "uniform")
        else ("configs[2] (B8 weak scaling)" if args.dist == "uniform" else "configs[3] (Z)"),
        "write_ratio_pct": args.write_ratio,
        "ops_per_gpu_per_round": args.ops_per_gpu,
        "put_responses": "Ok(None) as benches/hashmap.rs:114-119",
        "parallelism": "replicas%d" % world,
    })
    res["roofline"] = roofline("hm_round+hm_papply" if a_n else "hm_round",
                               round_bytes, k_n, k_ms, args,
                               measured_traffic(args), win)
    res["round"] = {
        "algorithmic_bytes": int(round_bytes),
        "achieved_GBps": round(round_bytes / (elapsed / args.steps) / 1e9, 1),
        "host_enqueue_us": round(host_s[0] * 1e6 / args.steps, 2),
        "host_first_steps_us": host_s[1:],
        "host_first_step_by_region_us": Env.first_calls,
        "distinct_get_keys": int(u_r),
        "distinct_put_keys": int(u_w),
    }
    if not args.partitioned:
        s = amdahl_speedup(world, args.write_ratio)
        res["amdahl"] = {"predicted_speedup_vs_1gpu": round(s, 3), "write_pct": args.write_ratio,
                         "c_w_over_c_r": 2.0,
                         "model": "SURVEY.md 8(e): S(G) = G(w c_w + (1-w) c_r) / (w c_w G + (1-w) c_r), "
                                  "all-gather time ignored; every replica replays every Put"}
    if prev_value is not None:
        res["variants"] = {"prev_value_responses_Mops": round(prev_value, 3)}
    if not args.no_cpu_baseline and world == 1 and args.dist == "uniform" and not args.partitioned:
        log(f"cpu baseline: {args.cpu_seconds}s ...")
        try:
            res["cpu_baseline"] = cpu_baseline(args.cpu_seconds, args.write_ratio, args.key_space, args.prefill)
        except Exception as e:  # noqa: BLE001
            res["cpu_baseline"] = {"error": str(e)}
    return res


# ---------------------------------------------------------------------------------------------
def _nr_groups(threads=None):
    """The thread budget spread over the NUMA nodes, one Replica per node (as _nr_cpu_run)."""
    cpus = sorted(os.sched_getaffinity(0))
    budget = cpu_budget(len(cpus)) if threads is None else threads
    nodes = numa_groups(cpus)
    per = max(1, budget // len(nodes))
    groups = [g[:per] for g in nodes][: max(1, min(len(nodes), budget))]
    cpu_list, rep = [], []
    for r, g in enumerate(groups):
        cpu_list += g
        rep += [r] * len(g)
    return cpu_list, rep, groups


def stack_cpu_baseline(seconds, n_ops, init):
    """The stack scale-out (benches/stack.rs:115-134) through the C++ restatement of nr: pinned
    threads on the job's CPU budget, one Replica per NUMA node, execute_mut(Push/Pop) from a
    shared 10,000-op stream, Stack::default (0..50000) per replica. Beside it, the sequential
    oracle Stack (a Vec in a loop, no log) on one core, labelled as such."""
    import numpy as np
    import oracle

    cpu_list, rep, groups = _nr_groups()
    r = oracle.nr_stack_bench(cpu_list, rep, seconds, 10_000, 0x5AC)
    out = {"value": round(r.ops / r.seconds / 1e6, 3), "unit": "Mops/s", "cores": len(cpu_list), "kind": "port",
           "sample": ("%.1f s of the stack scale-out (benches/stack.rs:115-134: 10,000-op 50/50 Push/Pop stream, "
                      "seeded) through the C++ restatement of nr (log + flat combining) on %d threads, %d replica(s) "
                      "(one per NUMA node); %d ops" % (r.seconds, len(cpu_list), len(groups), r.ops)),
           "host": host_topology()}
    side = min(3.0, seconds)
    t1 = oracle.nr_stack_bench(cpu_list[:1], [0], side, 10_000, 0x5AC)
    out["one_thread_nr"] = {"value": round(t1.ops / t1.seconds / 1e6, 3), "unit": "Mops/s", "cores": 1,
                            "sample": "the same stream through nr on 1 thread, 1 replica, %.1f s" % t1.seconds}
    st = oracle.Stack(np.arange(init, dtype=np.uint32))
    vals, ops = oracle.gen_stack_ops(n_ops, 0x5AC)
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < side:
        st.replay(vals, ops)
        done += n_ops
    el = time.perf_counter() - t0
    out["one_thread_sequential"] = {
        "value": round(done / el / 1e6, 3), "unit": "Mops/s", "cores": 1,
        "sample": "%.1f s of %d-op batches replayed by the sequential oracle Stack (no log, no combining)" % (el, n_ops)}
    return out


def synth_cpu_baseline(seconds, n_ops):
    """The synthetic scale-out (benches/synthetic.rs:296-335) through the C++ restatement of nr:
    ReadWrite ops from a shared 10,000-op stream, tid = the issuing thread's core id, 200,000
    CachePadded words per replica, one Replica per NUMA node. Beside it, the sequential oracle
    AbstractDataStructure on one core, labelled as such."""
    import numpy as np
    import oracle

    cpu_list, rep, groups = _nr_groups()
    r = oracle.nr_synth_bench(cpu_list, rep, seconds, 10_000, 0x5E7)
    out = {"value": round(r.ops / r.seconds / 1e6, 3), "unit": "Mops/s", "cores": len(cpu_list), "kind": "port",
           "sample": ("%.1f s of the synthetic scale-out (benches/synthetic.rs:296-335: 10,000 ReadWrite ops, tid = "
                      "core id, seeded r1/r2) through the C++ restatement of nr (log + flat combining) on %d "
                      "threads, %d replica(s) (one per NUMA node); %d ops" % (r.seconds, len(cpu_list), len(groups),
                                                                             r.ops)),
           "host": host_topology()}
    side = min(3.0, seconds)
    t1 = oracle.nr_synth_bench(cpu_list[:1], [0], side, 10_000, 0x5E7)
    out["one_thread_nr"] = {"value": round(t1.ops / t1.seconds / 1e6, 3), "unit": "Mops/s", "cores": 1,
                            "sample": "the same stream through nr on 1 thread, 1 replica, %.1f s" % t1.seconds}
    sy = oracle.Synthetic()
    raw = oracle.gen_raw(3 * n_ops, 0x5E7)
    ops = np.stack([raw[0::3] % 64, raw[1::3], raw[2::3], np.ones(n_ops, np.uint64)], axis=1)
    t0 = time.perf_counter()
    done = 0
    while time.perf_counter() - t0 < side:
        sy.replay(ops)
        done += n_ops
    el = time.perf_counter() - t0
    out["one_thread_sequential"] = {
        "value": round(done / el / 1e6, 3), "unit": "Mops/s", "cores": 1,
        "sample": "%.1f s of %d-op ReadWrite batches replayed by the sequential oracle (no log, no combining)" % (
            el, n_ops)}
    return out


def run_synthetic(args, env):
    """AbstractDataStructure log replay (benches/synthetic.rs:60-195, ReadWrite only as the
    bench issues, :302,316): rounds of N ops per GPU, each ReadWrite = 1 hot + 5 cold touches
    of a 200,000-word storage."""
    torch = env.torch
    import nrgpu
    from nrgpu import _lib as L

    world, rank, dev_t = env.world, env.rank, env.dev
    N = args.ops_per_gpu
    Ng = N * world
    rep = nrgpu.DeviceReplica(L.NRG_DS_SYNTHETIC, env.local, max_batch=Ng, log_bytes=64 * 4 * max(Ng, 8192),
                              replica_id=rank + 1, pipeline=args.pipeline)
    apply_knobs(rep, args)
    rep.use_torch_stream()
    P = max(1, min(args.pool, 8, args.steps + args.warmup))
    gen = torch.Generator(device=dev_t)
    gen.manual_seed(0x53594E54 + rank)
    lo, hi = -(1 << 63), (1 << 63) - 1
    ops = torch.empty((P, N, 4), dtype=torch.int64, device=dev_t)
    for p in range(P):  # {tid, r1, r2, op}: tid = a core id < 64, op = ReadWrite
        ops[p, :, 0] = torch.randint(0, 64, (N,), generator=gen, device=dev_t)
        ops[p, :, 1] = torch.randint(lo, hi, (N,), generator=gen, device=dev_t)
        ops[p, :, 2] = torch.randint(lo, hi, (N,), generator=gen, device=dev_t)
        ops[p, :, 3] = 1
    # pipeline=1: a round's sums are written in the next round's first launch, so rounds
    # alternate between two response buffers
    resps = [torch.empty(N, dtype=torch.int64, device=dev_t) for _ in range(2)]
    somes = [torch.empty(N, dtype=torch.uint8, device=dev_t) for _ in range(2)]
    torch.cuda.synchronize()
    group = cgroup = None
    if world > 1 and args.backend == "nccl":
        from nrgpu.parallel import ReplicaGroup

        WATCH.phase = "nrg_group_join"
        cgroup = ReplicaGroup(rep, rank, world, timeout_ms=args.group_timeout_ms)
        inputs = torch.cuda.Stream(dev_t)
        cgroup.set_input_stream(inputs.cuda_stream)
    elif world > 1:
        from nrgpu.parallel import ReplicatedLog

        group = ReplicatedLog(rep, device=dev_t)
    round_fn, h = rep._lib.nrg_synth_round_async, rep._h
    ptrs = [ops[p].data_ptr() for p in range(P)]
    rps = [(r.data_ptr(), s_.data_ptr()) for r, s_ in zip(resps, somes)]
    gathered = {}
    mode = {"n": 0}
    seg_lens = [N] * world

    def step(i):
        p = i % P
        r_p, s_p = rps[i & 1]
        if cgroup is not None:
            cgroup.round_async(ptrs[p], N, r_p, s_p, seg_lens=seg_lens)
        elif group is None:
            # Replica::combine of the batch: Log::append fused into the partition pass
            rc = round_fn(h, ptrs[p], N, rank + 1, r_p, s_p)
            if rc:
                L.check(rc, "synthetic round")
        else:
            g = gathered.pop(i) if i in gathered else group.gather_async(ops[p], stride=N)
            if i + 1 < mode["n"]:
                gathered[i + 1] = group.gather_async(ops[(i + 1) % P], stride=N)
            group.replay(g, resps[i & 1], somes[i & 1])

    mode["n"] = args.warmup
    for i in range(args.warmup):
        step(i)
    rep.sync()
    def run(n, evs=None):
        mode["n"] = n
        return env.timed(n, step, rep, evs=evs)

    WATCH.phase = "timed region"
    elapsed = run(args.steps)  # no events in the timed region
    kt, win = roofline_region(args, rep, run, ["sy_replay"])
    k_n, k_ms = kt["sy_replay"]
    rep.sync()
    value = world * N * args.steps / elapsed / 1e6
    if rank != 0:
        return None
    # B = 32 N + 2 * 8 * 200,000 per replica per batch (records; storage read and
    # written once, L2-resident); touches are reported beside it
    round_bytes = 32 * Ng + 2 * 8 * 200_000
    res = common_fields(args, env, value, elapsed * 1e3 / args.steps,
                        "Mops/s whole node, synthetic AbstractDataStructure log replay (benches/synthetic.rs)",
                        "u64", {
                            "workload": ("AbstractDataStructure replica per GPU: 200,000 words, rounds of %d ReadWrite "
                                         "ops/GPU (tid < 64, random r1/r2), sums for own ops%s" % (
                                             N, "; op segments all-gathered, every replica replays all %d ops" % Ng
                                             if world > 1 else "")),
                            "ops_per_gpu_per_round": N,
                            "parallelism": "replicas%d" % world,
                        })
    res["roofline"] = roofline("sy_replay", round_bytes, k_n, k_ms, args, measured_traffic(args), win)
    res["round"] = {"algorithmic_bytes": int(round_bytes),
                    "touches_per_s": round(6 * Ng * args.steps / elapsed, 1)}
    if not args.no_cpu_baseline and world == 1:
        res["cpu_baseline"] = synth_cpu_baseline(min(args.cpu_seconds, 10.0), min(N, 1 << 20))
    return res


def run_stack(args, env):
    torch = env.torch
    import nrgpu
    from nrgpu import _lib as L

    world, rank, dev_t = env.world, env.rank, env.dev
    N = args.ops_per_gpu
    Ng = N * world
    cap = args.stack_init + 4 * Ng + (1 << 16)
    rep = nrgpu.DeviceReplica(L.NRG_DS_STACK, env.local, max_batch=Ng, stack_capacity=cap,
                              log_bytes=64 * 4 * max(Ng, 8192), replica_id=rank + 1, pipeline=args.pipeline)
    apply_knobs(rep, args)
    rep.use_torch_stream()
    rep.st_init(list(range(args.stack_init)))  # benches/stack.rs:50-63: 0..50000
    P = max(1, min(args.pool, args.steps + args.warmup))
    ops = torch.empty((P, N), dtype=torch.int64, device=dev_t)
    seed0 = 0x5354434B00000001 + rank * 0x1000193
    for p in range(P):
        rep.gen_stack_ops_device(ops[p], N, seed0 + p)
    # pipeline=1: a round's cross-tile Pops are answered in the next round's launch, so rounds
    # alternate between two response buffers
    resps = [torch.empty(N, dtype=torch.int32, device=dev_t) for _ in range(2)]
    somes = [torch.empty(N, dtype=torch.uint8, device=dev_t) for _ in range(2)]
    resp, some = resps[0], somes[0]
    torch.cuda.synchronize()
    # distinct slots written per round (S of SURVEY.md §8d): pushes at distinct depths; the
    # depth walk is shift-invariant while it stays above 0 (it starts at 50k)
    S = 0
    for p in range(min(P, 4)):
        o = ops[p]
        push = (o >> 32) & 1
        step_d = push * 2 - 1
        d_before = torch.cumsum(step_d, 0) - step_d
        S += int(torch.unique(d_before[push == 1]).numel())
    S = S / min(P, 4) * world

    group = cgroup = None
    if world > 1 and args.backend == "nccl":
        from nrgpu.parallel import ReplicaGroup

        WATCH.phase = "nrg_group_join"
        cgroup = ReplicaGroup(rep, rank, world, timeout_ms=args.group_timeout_ms)
        inputs = torch.cuda.Stream(dev_t)
        cgroup.set_input_stream(inputs.cuda_stream)
    elif world > 1:
        from nrgpu.parallel import ReplicatedLog

        group = ReplicatedLog(rep, device=dev_t)
    round_fn, h = rep._lib.nrg_stack_round_async, rep._h
    ptrs = [ops[p].data_ptr() for p in range(P)]
    rps = [(r.data_ptr(), s_.data_ptr()) for r, s_ in zip(resps, somes)]
    gathered = {}
    mode = {"n": 0}
    seg_lens = [N] * world

    def step(i):
        p = i % P
        r_p, s_p = rps[i & 1]
        if cgroup is not None:
            cgroup.round_async(ptrs[p], N, r_p, s_p, seg_lens=seg_lens)
        elif group is None:
            # Replica::combine of the batch: Log::append fused into the replay pass
            rc = round_fn(h, ptrs[p], N, rank + 1, r_p, s_p)
            if rc:
                L.check(rc, "stack round")
        else:
            g = gathered.pop(i) if i in gathered else group.gather_async(ops[p], stride=N)
            if i + 1 < mode["n"]:
                gathered[i + 1] = group.gather_async(ops[(i + 1) % P], stride=N)
            group.replay(g, resps[i & 1], somes[i & 1])

    mode["n"] = args.warmup
    for i in range(args.warmup):
        step(i)
    rep.sync()
    def run(n, evs=None):
        mode["n"] = n
        return env.timed(n, step, rep, evs=evs)

    WATCH.phase = "timed region"
    elapsed = run(args.steps)  # no events in the timed region
    kt, win = roofline_region(args, rep, run, ["st_replay"])
    k_n, k_ms = kt["st_replay"]
    rep.sync()
    value = world * N * args.steps / elapsed / 1e6
    if rank != 0:
        return None
    # B = 8 N + 4 N + 4 S per replica per round (records, responses, slots written)
    round_bytes = 8 * Ng + 4 * N + 4 * S
    res = common_fields(args, env, value, elapsed * 1e3 / args.steps,
                        "Mops/s whole node, Stack push/pop log replay (benches/stack.rs)", "u32", {
                            "workload": ("Stack replica per GPU: initial %d elements, rounds of %d ops/GPU (50/50 "
                                         "push/pop, seeded), pop responses for own ops%s" % (
                                             args.stack_init, N, "; op segments all-gathered, every replica "
                                             "replays all %d ops" % Ng if world > 1 else "")),
                            "baseline_config": "configs[4] (S1/S8)",
                            "ops_per_gpu_per_round": N,
                            "parallelism": "replicas%d" % world,
                        })
    res["roofline"] = roofline("st_replay", round_bytes, k_n, k_ms, args, measured_traffic(args), win)
    res["round"] = {"algorithmic_bytes": int(round_bytes), "distinct_slots_written": int(S)}
    if not args.no_cpu_baseline and world == 1:
        res["cpu_baseline"] = stack_cpu_baseline(min(args.cpu_seconds, 10.0), N, args.stack_init)
    return res


def write_scaleout_csv(path, name, world, ops_per_rank_per_round, steps, elapsed):
    """Append rows in the reference harness's scaleout_benchmarks.csv format
    (benches/mkbench.rs:498-552: name, rs, tm, batch_size, threads, duration, thread_id, core_id,
    exp_time_in_sec, iterations), so CPU and GPU results plot with the reference's tooling
    (benches/hashbench_plot.r). One row per GPU replica: rs = "GPU" (one replica per GPU, the
    analogue of ReplicaStrategy::Socket per NUMA node), thread_id = core_id = rank, and the
    per-second counter `iterations` = that replica's ops per second over the timed region (the
    region is far shorter than the reference's 1-s sampling interval)."""
    import csv

    new = not os.path.exists(path)
    with open(path, "a", newline="") as f:
        w = csv.writer(f)
        if new:
            w.writerow(["name", "rs", "tm", "batch_size", "threads", "duration", "thread_id", "core_id",
                        "exp_time_in_sec", "iterations"])
        for r in range(world):
            w.writerow([name, "GPU", "Sequential", ops_per_rank_per_round, world, round(elapsed, 6), r, r, 1,
                        int(ops_per_rank_per_round * steps / elapsed)])


def _free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv, script=None):
    """`python3 bench.py --gpus N` without a launcher: start N rank processes of this script, one
    per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set as torch.distributed.run sets them),
    relay rank 0's JSON line, and return non-zero if any rank fails or the deadline passes. The
    reference's harness likewise spawns its own workers per replica (benches/mkbench.rs:611-700,
    benches/hashmap.rs:226-259). This parent process makes no GPU call: no torch, no libnrgpu."""
    import subprocess

    n = args.gpus
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL across processes)
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    log(f"launched {n} ranks (pids {[p.pid for p in procs]}), rendezvous 127.0.0.1:{port}")
    lines = []
    reader = threading.Thread(target=lambda: lines.extend(procs[0].stdout.read().decode().splitlines()),
                              daemon=True)
    reader.start()
    deadline = time.monotonic() + (args.deadline if args.deadline > 0 else float("inf")) + 30.0
    status = 0
    while True:
        codes = [p.poll() for p in procs]
        failed = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if failed:
            r, c = failed[0]
            log(f"rank {r} exited with status {c}; stopping the other ranks")
            status = c if c > 0 else 1
            break
        if all(c == 0 for c in codes):
            break
        if time.monotonic() > deadline:
            log(f"ranks {[r for r, c in enumerate(codes) if c is None]} still running past the deadline; stopping")
            status = 3
            break
        time.sleep(0.05)
    if status:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    reader.join(timeout=10)
    if status == 0:
        out = [ln for ln in lines if ln.startswith("{")]
        if not out:
            log("rank 0 printed no result line")
            return 1
        print(out[-1], flush=True)
    return status


def amdahl_speedup(n, write_pct, cw_over_cr=2.0):
    """whole-node speedup of full replication over one replica,
    S(G) = G (w c_w + (1-w) c_r) / (w c_w G + (1-w) c_r), the all-gather ignored. c_w / c_r = 2
    is calibrated from the per-GPU emulated rounds (100k Puts + 900k Gets in 34.3 us,
    800k + 900k in 79 us)."""
    w = write_pct / 100.0
    a = cw_over_cr
    return n * (w * a + (1 - w)) / (w * a * n + (1 - w))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--workload", default="hashmap", choices=["hashmap", "stack", "synthetic"])
    ap.add_argument("--write-ratio", type=int, default=10)
    ap.add_argument("--ops-per-gpu", type=int, default=1_000_000)
    ap.add_argument("--key-space", type=int, default=10_000_000)
    ap.add_argument("--dist", default="uniform", choices=["uniform", "zipf"])
    ap.add_argument("--theta", type=float, default=0.99)
    ap.add_argument("--scramble", action="store_true", help="Zipf: key = mix64(rank) %% N (hot keys spread)")
    ap.add_argument("--prefill", type=int, default=1 << 23)
    ap.add_argument("--log2-slots", type=int, default=26)
    ap.add_argument("--stack-init", type=int, default=50_000)
    ap.add_argument("--partitioned", action="store_true",
                    help="hashmap: cnr-style key-partitioned rounds (SURVEY.md 8 f4) instead of full replication")
    ap.add_argument("--pool", type=int, default=64, help="distinct pre-generated input batches")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-prev-variant", action="store_true")
    ap.add_argument("--opening", choices=["sync", "spin", "keep"], default="spin",
                    help="how the timed region's opening sync waits: polled with the host thread awake, then "
                         "torch.cuda.synchronize (default; profiles/r05_opening_ab.txt), or the plain sync alone")
    ap.add_argument("--no-kernel-timing", action="store_true", help="diagnostic: no HIP events in the timed region")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo: CPU rehearsal)")
    ap.add_argument("--share-gpu", action="store_true", help="all ranks on cuda:0 (gloo rehearsal on a 1-GPU box)")
    ap.add_argument("--csv", default=None, help="append scaleout_benchmarks.csv rows (reference format)")
    ap.add_argument("--timing-every", type=int, default=4,
                    help="roofline region: event-stamp every n-th launch of the dominant kernel (>= 16 samples "
                         "over its 64+ rounds; the timed region itself is never stamped)")
    ap.add_argument("--knob", action="append", default=[], metavar="NAME=VALUE",
                    help="diagnostic/tuning knob of the replica (nrg_test_set_knob, include/nrgpu_testing.h), "
                         "e.g. K1=2; never needed for the headline")
    ap.add_argument("--deadline", type=float, default=900.0,
                    help="whole-process watchdog in seconds (0: off): a stalled rank exits 3 with a diagnostic")
    ap.add_argument("--group-timeout-ms", type=int, default=120_000,
                    help="replica group deadline for every wait on the peer ranks (nrg_group_set_timeout)")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="1: a round's apply+reads ride in the next round's launch (nrg_config.pipeline); "
                         "0: every round call completes its own reads")
    args = ap.parse_args()
    args.timing_every = max(1, args.timing_every)
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    ws = os.environ.get("WORLD_SIZE")
    if ws is None and args.gpus > 1:
        # no launcher around us: start the N ranks ourselves (this process never touches the GPU)
        sys.exit(launch_ranks(args, sys.argv[1:]))
    if ws is not None and int(ws) != args.gpus:
        log(f"WORLD_SIZE={ws} but --gpus={args.gpus}: refusing to measure a different GPU count than asked")
        sys.exit(2)
    WATCH.arm(args.deadline)
    env = Env(args)
    runner = {"stack": run_stack, "synthetic": run_synthetic}.get(args.workload, run_hashmap)
    res = runner(args, env)
    if res is not None:
        if args.csv:
            name = {"stack": "nrstack-gpu", "synthetic": "nrsynthetic-gpu"}.get(
                args.workload, "nrhashmap-gpu-wr%d-%s" % (args.write_ratio, key_dist_name(args)))
            write_scaleout_csv(args.csv, name, env.world, args.ops_per_gpu, args.steps,
                               res["ms_per_step"] * args.steps / 1e3)
        print(json.dumps(res), flush=True)
    env.close()


if __name__ == "__main__":
    main()
