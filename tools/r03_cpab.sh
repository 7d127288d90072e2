#!/bin/bash
set -euo pipefail
bash tools/ab_suite_prof.sh r03_cpab "c3_mixed str_dict c4_lineitem" abx/libcur.so abx/libcp32.so abx/libcp24.so
for l in libcur libcp32 libcp24; do echo "== $l"; python3 tools/seg_kernels.py gpurun_out/r03_cpab/$l/run_kernel_trace.csv --names c3,str_dict,c4_8M | grep -E "^\[|bin_copy" || true; done
