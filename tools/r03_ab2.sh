#!/bin/bash
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_zdiag
PQGPU_LIB=$PWD/abx/libzdiag.so timeout -k 10 300 python3 -u tools/diag_zstd.py > gpurun_out/r03_zdiag/diag.txt 2>&1 || { tail -20 gpurun_out/r03_zdiag/diag.txt; exit 1; }
cat gpurun_out/r03_zdiag/diag.txt
bash tools/ab_suite_prof.sh r03_ab2 "c3_mixed str_plain str_dict c4_lineitem" abx/libcp512.so abx/libcp1024.so abx/libcp256.so
