"""Per-kernel averages of rocprofv3 --pmc passes (counter_collection.csv files under a directory):
prints, per kernel name, every counter's mean per dispatch (summed over the dispatch's dimensions),
then the derived issue figures (MI355X_MICROARCH.md: a wave64 VALU instruction takes its SIMD-32 2
cycles; SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles; GRBM_GUI_ACTIVE summed over
the 8 XCDs, so the dispatch's cycles are GRBM_GUI_ACTIVE / 8):
  valu_util  = 2 x SQ_INSTS_VALU / (1024 SIMDs x cycles)   (issue share of every SIMD's VALU)
  salu_util  = SQ_INSTS_SALU / (256 CUs x cycles)           (one scalar instruction per CU per cycle)
  wait_frac  = SQ_WAIT_ANY / SQ_WAVE_CYCLES                 (wave-cycles spent waiting on a dependency)
  issue_frac = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES"""
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
    mean = {}
    for cn in sorted(per[k]):
        vals = per[k][cn]
        mean[cn] = sum(vals) / len(vals)
        print(f"   {cn:28s} {mean[cn]:18.1f}   ({len(vals)} dispatches)")
    cyc = mean.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    if cyc > 0:
        print(f"   {'cycles (GRBM_GUI_ACTIVE/8)':28s} {cyc:18.1f}")
        if "SQ_INSTS_VALU" in mean:
            print(f"   {'valu_util':28s} {2.0 * mean['SQ_INSTS_VALU'] / (1024.0 * cyc):18.3f}")
        if "SQ_INSTS_SALU" in mean:
            print(f"   {'salu_util':28s} {mean['SQ_INSTS_SALU'] / (256.0 * cyc):18.3f}")
    if mean.get("SQ_WAVE_CYCLES"):
        for num, name in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "wait_inst_frac"),
                          ("SQ_ACTIVE_INST_ANY", "issue_frac")):
            if num in mean:
                print(f"   {name:28s} {mean[num] / mean['SQ_WAVE_CYCLES']:18.3f}")
