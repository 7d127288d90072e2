#!/usr/bin/env python3
"""Per-workload kernel medians from a rocprofv3 kernel trace: dispatches are split into workloads at
host gaps longer than --gap seconds (input generation between suite workloads).
usage: python3 tools/seg_kernels.py <run_kernel_trace.csv> [--names w1,w2,...] [--top N]"""
import argparse
import collections
import csv

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--gap", type=float, default=0.5)
ap.add_argument("--names", default="")
ap.add_argument("--top", type=int, default=6)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
segs, last = [[]], None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if last is not None and s - last > a.gap * 1e9:
        segs.append([])
    segs[-1].append(r)
    last = e
names = a.names.split(",") if a.names else []
for i, sg in enumerate(segs):
    d = collections.defaultdict(list)
    for r in sg:
        if "pqg" in r["Kernel_Name"]:
            d[r["Kernel_Name"].split("(")[0].replace("void ", "")].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    if not d:
        continue
    print(f"[{names[i] if i < len(names) else i}]")
    for k, v in sorted(d.items(), key=lambda kv: -sorted(kv[1])[len(kv[1]) // 2])[: a.top]:
        v = sorted(v)
        print(f"   {k[:34]:34s} n={len(v):3d} median {v[len(v) // 2]:9.1f} us")
