#!/bin/bash
# C4 column groups solo under rocprofv3 kernel stats (diagnostics): bash tools/c4_prof_groups.sh <tag> <groups...>
set -euo pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
for g in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$g" -o run -- \
    python3 bench.py --workload c4 --rows 125000000 --steps 5 --warmup 1 --no-cpu --c4-cols $g > "$OUT/prof_$g.json" 2> "$OUT/prof_$g.err" \
    || { tail -20 "$OUT/prof_$g.err"; exit 1; }
  echo "== $g"; python3 tools/kstats.py "$OUT/prof_$g"
done
