#!/bin/bash
# Session: ZSTD (LDS length codes, inlined helpers) diag + parity + codec suite; then the string path
# (segmented walk, 512-value copy chunks) parity, suite and the C4 125M-row shard.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_zdiag2
PQGPU_LIB=$PWD/abx/libzdiag.so timeout -k 10 300 python3 -u tools/diag_zstd.py > gpurun_out/r03_zdiag2/diag.txt 2>&1 || { tail -20 gpurun_out/r03_zdiag2/diag.txt; exit 1; }
cat gpurun_out/r03_zdiag2/diag.txt
bash tools/r03_zstd.sh r03_zstd3
bash tools/r03_str.sh r03_str3
