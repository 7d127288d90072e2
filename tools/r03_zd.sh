#!/bin/bash
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_zd
PQGPU_LIB=$PWD/abx/libzdiag.so timeout -k 10 300 python3 -u tools/diag_zstd.py > gpurun_out/r03_zd/diag.txt 2>&1 || { tail -20 gpurun_out/r03_zd/diag.txt; exit 1; }
cat gpurun_out/r03_zd/diag.txt
