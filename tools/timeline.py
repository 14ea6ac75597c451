#!/usr/bin/env python3
"""Per-launch timeline of one kernel from a rocprofv3 kernel trace (run_kernel_trace.csv).

Prints, for launches [first, last) of kernels whose name contains NAME, the duration and the gap
to the previous launch of ANY kernel on the GPU (idle time between dispatches).
Usage: tools/timeline.py TRACE.csv NAME [first last]
"""
import csv
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    first = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    last = int(sys.argv[4]) if len(sys.argv) > 4 else 10 ** 9
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows))
    prev_end = None
    k = 0
    for s, e, n in ks:
        if name in n:
            if first <= k < last:
                gap = (s - prev_end) / 1e3 if prev_end is not None else float("nan")
                print(f"{k:4d} {n[:40]:40s} dur {(e - s) / 1e3:8.2f} us  gap {gap:8.2f} us")
            k += 1
        prev_end = e if prev_end is None else max(prev_end, e)


if __name__ == "__main__":
    main()
