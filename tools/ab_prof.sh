#!/bin/bash
# Kernel-level A/B: rocprofv3 --kernel-trace --stats of bench.py per variant.
#   bash tools/ab_prof.sh <tag> "<label>:<ENV=V ...>:<lib or default>" ...
# Prints each variant's kernels (avg us, calls). Stops at the first failure.
set -euo pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for spec in "$@"; do
  IFS=: read -r label envs lib <<< "$spec"
  if [ "$lib" = default ]; then unset PQGPU_LIB; else export PQGPU_LIB=$PWD/$lib; fi
  for e in $envs; do export "$e"; done
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$label" -o run -- python3 -u bench.py --no-cpu --no-verify \
    --steps 30 ${AB_ARGS:-} > "$OUT/$label.json" 2> "$OUT/$label.err" || { tail -20 "$OUT/$label.err"; exit 1; }
  for e in $envs; do unset "${e%%=*}"; done
  f=$(find "$OUT/$label" -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$label" "$OUT/$label.json" <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
b = json.load(open(sys.argv[3]))
print(f"== {sys.argv[2]}: bench {b['value']/1e9:.1f} G/s {b['ms_per_step']*1e3:.1f} us/step")
for r in rows:
    if int(r["Calls"]) >= 10:
        print(f"   {r['Name'][:70]:70s} avg {float(r['AverageNs'])/1e3:8.1f} us  min {float(r['MinNs'])/1e3:8.1f}  calls {r['Calls']}")
PY
done
