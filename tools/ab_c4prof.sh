#!/bin/bash
# Kernel times of one C4 column group under each library build (diagnostics):
#   bash tools/ab_c4prof.sh <tag> <group> lib1.so ... ("default" = the product library)
set -euo pipefail
TAG=$1; G=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename "$lib" .so)
  if [ "$lib" = default ]; then unset PQGPU_LIB; else export PQGPU_LIB=$PWD/$lib; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$n" -o run -- \
    python3 bench.py --workload c4 --rows 125000000 --steps 5 --warmup 1 --no-cpu --no-verify --c4-cols $G > "$OUT/$n.json" 2> "$OUT/$n.err" \
    || { tail -20 "$OUT/$n.err"; exit 1; }
  echo "== $n"; python3 tools/kstats.py "$OUT/$n" | grep -v 'k_bin_walk\|k_dd_bases'
done
