#!/usr/bin/env python3
"""Run bench.py under several settings (one subprocess each) and print a compact table.

Usage: tools/sweep.py 'NAME|ENV=V ENV2=V2|--bench --args' ...
(replica tuning knobs are bench.py arguments: --knob K1=2 --knob PART=2; --with-prev also runs
the previous-value variant and prints its rate)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    base = ["--no-cpu-baseline", "--no-prev-variant", "--steps", "200"]
    for spec in sys.argv[1:]:
        name, envs, args = (spec.split("|") + ["", ""])[:3]
        env = dict(os.environ)
        for kv in envs.split():
            k, v = kv.split("=", 1)
            env[k] = v
        a = args.split()
        b = list(base)
        if "--with-prev" in a:
            a.remove("--with-prev")
            b.remove("--no-prev-variant")
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + b + a
        try:
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
        except subprocess.TimeoutExpired:
            print(f"{name:28s} TIMEOUT", flush=True)
            return 1
        if p.returncode != 0:
            print(f"{name:28s} FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
            return 1
        d = json.loads(p.stdout.strip().splitlines()[-1])
        r = d["roofline"]
        print(f"{name:28s} {d['value']:10.1f} Mops/s  {d['ms_per_step'] * 1e3:8.2f} us/round  "
              f"kernel {r['avg_launch_us']} us x{r['launches']}  frac {r['frac']}  host {d['round'].get('host_enqueue_us')} us"
              + (f"  prev {d['variants']['prev_value_responses_Mops']} Mops/s" if "variants" in d else ""), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
