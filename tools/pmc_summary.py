"""Summarize tools/pmc.sh output: per-kernel average of each counter per dispatch."""
import collections, csv, glob, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/pass*/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "pqg::" not in name:
            continue
        per[(name.split("(")[0], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, d, c), v in per.items():
        acc[k][c].append(v)
for k, cs in acc.items():
    print(k)
    for c, vs in sorted(cs.items()):
        print(f"   {c:28s} {sum(vs)/len(vs):16.1f}")
