#!/bin/bash
# ZSTD: cycles per sequence with 1 wave per CU (grid 256), 1 per SIMD (1024), default (4096).
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_zgrid
for v in libzdiag256 libzdiag1024 libzdiag; do
  PQGPU_LIB=$PWD/abx/$v.so timeout -k 10 300 python3 -u tools/diag_zstd.py > gpurun_out/r03_zgrid/$v.txt 2>&1 || { tail -20 gpurun_out/r03_zgrid/$v.txt; exit 1; }
  echo "== $v"; tail -3 gpurun_out/r03_zgrid/$v.txt
done
