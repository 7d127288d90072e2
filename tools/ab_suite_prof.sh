#!/bin/bash
# Per-kernel times of suite workloads per library: bash tools/ab_suite_prof.sh <tag> "<workloads>" lib1.so lib2.so ...
set -euo pipefail
TAG=$1; shift
WL=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for lib in "$@"; do
  n=$(basename "$lib" .so)
  export PQGPU_LIB=$PWD/$lib
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$n" -o run -- \
    python3 -u tools/bench_suite.py $WL --cpu-budget 0 --steps 5 --warmup 1 > "$OUT/$n.jsonl" 2> "$OUT/$n.err" \
    || { tail -20 "$OUT/$n.err"; exit 1; }
  f=$(find "$OUT/$n" -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$n" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print("==", sys.argv[2])
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    if "pqg" in r["Name"]:
        print(f"   {r['Name'].split('(')[0][:50]:50s} avg {float(r['AverageNs'])/1e3:9.1f} us  calls {r['Calls']}")
PY
done
