#!/bin/bash
# C2 ramp study: walker phase timeline (diagnostic build), then walker priority / expansion order A/B.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_c2ab
PQGPU_LIB=$PWD/abx/libdiag.so timeout -k 10 300 python3 -u tools/diag_fused.py 1.5 gpurun_out/r03_c2ab/diag_c2.json \
  > gpurun_out/r03_c2ab/diag.txt 2>&1 || { tail -20 gpurun_out/r03_c2ab/diag.txt; exit 1; }
cat gpurun_out/r03_c2ab/diag.txt
bash tools/ab_bench.sh r03_c2ab default abx/libprio.so abx/liborder.so abx/libboth.so
AB_ARGS="--zipf 2.0" bash tools/ab_bench.sh r03_c2ab_z2 default abx/libprio.so abx/liborder.so abx/libboth.so
bash tools/ab_suite_prof.sh r03_segab "c3_mixed c4_lineitem" abx/libcur.so abx/libsegall.so
