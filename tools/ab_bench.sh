#!/bin/bash
# A/B of library builds on the C2 bench: bash tools/ab_bench.sh <tag> lib1.so lib2.so ...
# ("default" = parquet-mr_amd/pqgpu/libpqgpu.so; AB_ARGS adds bench.py flags). Each run has its own time limit; stops on failure.
set -euo pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    if [ "$lib" = default ]; then unset PQGPU_LIB; else export PQGPU_LIB=$PWD/$lib; fi
    timeout -k 10 180 python -u bench.py --no-cpu --steps 50 ${AB_ARGS:-} > "$OUT/$n.$rep.json" 2> "$OUT/$n.$rep.err" \
      || { tail -20 "$OUT/$n.$rep.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e9,1), 'G/s', round(d['ms_per_step']*1e3,1), 'us')" "$OUT/$n.$rep.json" "$n"
  done
done
