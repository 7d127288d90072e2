#!/bin/bash
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_bpd2
PQGPU_LIB=$PWD/abx/libdiag.so timeout -k 10 300 python3 -u tools/diag_binplain.py str_plain > gpurun_out/r03_bpd2/str_plain.txt 2>&1 || { tail -20 gpurun_out/r03_bpd2/str_plain.txt; exit 1; }
cat gpurun_out/r03_bpd2/str_plain.txt
bash tools/ab_suite_prof.sh r03_bpd2 "c3_mixed str_plain c4_lineitem" abx/libclassic.so
python3 tools/seg_kernels.py gpurun_out/r03_bpd2/libclassic/run_kernel_trace.csv --names c3,str_plain,c4_8M || true
