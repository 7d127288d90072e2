#!/bin/bash
# A/B of library builds on suite workloads: bash tools/ab_suite.sh <tag> "<workloads>" lib1.so lib2.so ...
# Each run has its own time limit; stops on failure. SUITE_ARGS adds bench_suite.py flags.
set -euo pipefail
TAG=$1; shift
WL=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for lib in "$@"; do
  n=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset PQGPU_LIB; else export PQGPU_LIB=$PWD/$lib; fi
  timeout -k 10 400 python -u tools/bench_suite.py $WL --cpu-budget 0 ${SUITE_ARGS:-} > "$OUT/$n.jsonl" 2> "$OUT/$n.err" \
    || { tail -20 "$OUT/$n.err"; exit 1; }
  python3 - "$OUT/$n.jsonl" "$n" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(sys.argv[2], d["workload"], round(d["ms_per_launch"], 3), "ms", round(d["hbm_frac"], 3))
PY
done
