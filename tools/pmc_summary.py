"""Summarize separate rocprofv3 --pmc passes: per-kernel average of each counter per dispatch.

With --json OUT it also writes the HBM traffic per dispatch of every pqg:: kernel, corrected
as MI355X_MICROARCH.md (HBM section) prescribes for gfx950: FETCH_SIZE and WRITE_SIZE are in
KiB; FETCH_SIZE counts half of the bytes of wide (16 B/lane) streaming reads, so it is doubled;
WRITE_SIZE reads exactly for 16 B/lane streaming stores. bench.py reports that number as
roofline.traffic for its dominant kernel.
"""
import argparse
import collections
import csv
import glob
import json

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--json")
args = ap.parse_args()

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(args.dir + "/pass*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "pqg::" not in name:
            continue
        per[(name.split("(")[0], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, d, c), v in per.items():
        acc[k][c].append(v)
out = {}
for k, cs in acc.items():
    print(k)
    avg = {c: sum(vs) / len(vs) for c, vs in cs.items()}
    for c, v in sorted(avg.items()):
        print(f"   {c:28s} {v:16.1f}")
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        fetch = 2.0 * avg["FETCH_SIZE"] * 1024.0
        write = avg["WRITE_SIZE"] * 1024.0
        out[k] = {"fetch_bytes": fetch, "write_bytes": write, "traffic_bytes": fetch + write,
                  "counters": avg, "dispatches": len(cs["FETCH_SIZE"])}
        print(f"   HBM traffic per dispatch (FETCH x2 + WRITE): {(fetch + write) / 1e6:.1f} MB")
if args.json:
    json.dump(out, open(args.json, "w"), indent=1)
