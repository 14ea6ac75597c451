#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof_<tag>/) into profiles/<name>.txt.

Per kernel: launches and average duration from the kernel-trace stats, and the average
FETCH_SIZE / WRITE_SIZE per launch from the PMC passes, and (profile.sh ATOMIC=1) atomics at the
L2, atomics sent to memory and memory read requests per launch. gfx950 correction (MI355X_MICROARCH.md,
HBM section): FETCH_SIZE counts 128-B memory-side requests at 64 B, so it is doubled here;
WRITE_SIZE is taken as reported. Both counters are in KB.

Usage: tools/prof_summary.py gpurun_out/prof_<tag> profiles/<name>.txt
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").strip()


def one(pattern):
    m = sorted(glob.glob(pattern, recursive=True))
    return m[0] if m else None


def pmc(path, counter):
    """per kernel: (launches, MEDIAN value per launch) -- the median, so that the few partial
    launches of a timed region (its first launch, the join's flush launches) do not pull the
    per-round figure down"""
    acc = defaultdict(list)
    if not path:
        return {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row.get("Counter_Name") != counter:
                continue
            acc[short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return {k: (len(v), sorted(v)[len(v) // 2]) for k, v in acc.items()}


def main():
    d, out = sys.argv[1], sys.argv[2]
    stats = one(os.path.join(d, "trace", "**", "*kernel_stats.csv"))
    fetch = pmc(one(os.path.join(d, "fetch", "**", "*counter_collection.csv")), "FETCH_SIZE")
    write = pmc(one(os.path.join(d, "write", "**", "*counter_collection.csv")), "WRITE_SIZE")
    apath = one(os.path.join(d, "atomic", "**", "*counter_collection.csv"))
    atom = {c: pmc(apath, c) for c in ("TCC_ATOMIC_sum", "TCC_EA0_ATOMIC_sum", "TCC_EA0_RDREQ_sum")}
    lines = []
    bench = os.path.join(d, "bench_trace.json")
    if os.path.exists(bench):
        with open(bench) as f:
            txt = f.read().strip().splitlines()
        if txt:
            lines.append("bench line (under kernel trace): " + txt[-1])
            try:
                b = json.loads(txt[-1])
                lines.append("workload: %s" % b["config"]["workload"])
            except (ValueError, KeyError):
                pass
    lines.append("")
    hdr = ("kernel", "calls", "avg_us", "min_us", "FETCHx2_KB/l", "WRITE_KB/l")
    if apath:
        hdr += ("L2_ATOM/l", "EA_ATOM/l", "EA_RDREQ/l")
    lines.append(("%-28s %8s %11s %11s %14s %14s" + " %12s" * (len(hdr) - 6)) % hdr)
    if stats:
        with open(stats) as f:
            rows = list(csv.DictReader(f))
        for r in rows:
            k = short(r["Name"])
            fe = fetch.get(k)
            wr = write.get(k)
            line = "%-28s %8s %11.3f %11.3f %14s %14s" % (
                k[:28], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3,
                "%.1f" % (2 * fe[1]) if fe else "-", "%.1f" % wr[1] if wr else "-")
            if apath:
                for c in ("TCC_ATOMIC_sum", "TCC_EA0_ATOMIC_sum", "TCC_EA0_RDREQ_sum"):
                    v = atom[c].get(k)
                    line += " %12s" % ("%.0f" % v[1] if v else "-")
            lines.append(line)
    # HBM traffic per launch of the round kernel, for bench.py's roofline.traffic
    tk = None
    try:
        tk = json.loads(txt[-1])["roofline"].get("traffic_key")
    except (NameError, ValueError, KeyError, IndexError):
        pass
    # the timed unit: one hm_round launch, one stack round (st_round: tile pass of chunk e +
    # finish of chunk e-1) or one synthetic round (sy_part with the previous sums + sy_bucket)
    if tk and tk.startswith("stack"):
        parts = ["st_round_kernel"]
    elif tk and tk.startswith("synthetic"):  # one launch per round (sy_round), or two
        parts = ["sy_round_kernel"] if any("sy_round_kernel" in k for k in fetch) else ["sy_part_kernel", "sy_bucket_kernel"]
    else:  # a partition round adds its apply launch
        parts = ["hm_round_kernel"] + (["hm_papply_kernel"] if any("hm_papply" in k for k in fetch) else [])

    def per_unit(tab):
        got = [next((v for k, v in tab.items() if p in k), None) for p in parts]
        if any(g is None for g in got):
            return None
        return (got[0][0], sum(g[1] for g in got))

    fe, wr = per_unit(fetch), per_unit(write)
    if tk and fe and wr:
        tpath = os.path.join(os.path.dirname(os.path.abspath(out)), "traffic_hm_round.json")
        try:
            with open(tpath) as f:
                tj = json.load(f)
        except (OSError, ValueError):
            tj = {}
        tj[tk] = {"bytes_per_launch": int((2 * fe[1] + wr[1]) * 1024), "fetch_x2_bytes": int(2 * fe[1] * 1024),
                  "write_bytes": int(wr[1] * 1024), "launches": fe[0], "source": os.path.basename(out)}
        with open(tpath, "w") as f:
            json.dump(tj, f, indent=1, sort_keys=True)
        lines.append("traffic per " + "+".join(parts) + " launch: %.1f MB (FETCH_SIZE x2 %.1f MB + WRITE_SIZE %.1f MB) -> %s" % (
            (2 * fe[1] + wr[1]) * 1024 / 1e6, 2 * fe[1] * 1024 / 1e6, wr[1] * 1024 / 1e6, tpath))
    text = "\n".join(lines) + "\n"
    with open(out, "w") as f:
        f.write(text)
    print(text)


if __name__ == "__main__":
    main()
