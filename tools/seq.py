#!/usr/bin/env python3
"""Every dispatch in a window of a rocprofv3 kernel trace, in start order: name, duration and the
idle gap before it (diagnostic for multi-launch rounds). Usage: tools/seq.py TRACE.csv FIRST COUNT"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first, count = int(sys.argv[2]), int(sys.argv[3])
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")) for r in rows)
prev = None
for i, (s, e, n) in enumerate(ks):
    if first <= i < first + count:
        gap = (s - prev) / 1e3 if prev is not None else float("nan")
        print(f"{i:5d} {n[:56]:56s} dur {(e - s) / 1e3:8.2f} us  gap {gap:8.2f} us")
    prev = e if prev is None else max(prev, e)
print("total dispatches", len(ks))
