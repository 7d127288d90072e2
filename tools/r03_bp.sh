#!/bin/bash
# k_bin_plain timing: workgroup-order tiles (current) vs the same without the look-back (diagnostic).
set -euo pipefail
bash tools/ab_suite_prof.sh r03_bp "str_plain c3_mixed" abx/libcur.so abx/libnolb.so
for l in libcur libnolb; do echo "== $l"; python3 tools/seg_kernels.py gpurun_out/r03_bp/$l/run_kernel_trace.csv --names str_plain,c3 || true; done
