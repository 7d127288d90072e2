"""Per-kernel averages of rocprofv3 --pmc passes (counter_collection.csv files under a directory):
prints, per kernel name, every counter's mean per dispatch (summed over the dispatch's dimensions)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    acc = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
        acc[key] += float(r["Counter_Value"])
        names[key[0]] = r["Kernel_Name"].split("(")[0]
    for (disp, cn), v in acc.items():
        per[names[disp]][cn].append(v)
for k in sorted(per):
    if not k.startswith("pqg") and "pqg::" not in k:
        continue
    print(k)
    for cn in sorted(per[k]):
        vals = per[k][cn]
        print(f"   {cn:28s} {sum(vals) / len(vals):18.1f}   ({len(vals)} dispatches)")
