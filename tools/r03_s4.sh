#!/bin/bash
# Session: ZSTD lean sequence loop (diag + parity + suite), dictionary quarter chunks (parity), C2 walk
# phase counters, C2 tail-split A/B.
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03_s4
PQGPU_LIB=$PWD/abx/libzdiag.so timeout -k 10 300 python3 -u tools/diag_zstd.py > gpurun_out/r03_s4/zdiag.txt 2>&1 || { tail -20 gpurun_out/r03_s4/zdiag.txt; exit 1; }
tail -4 gpurun_out/r03_s4/zdiag.txt
bash tools/r03_zstd.sh r03_s4/zstd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_timeout.py tests/test_gpu_error_epochs.py tests/test_gpu_fixtures.py "tests/test_gpu_fullsize.py::test_c2_fresh_plan_first_launch" "tests/test_gpu_fullsize.py::test_c2_many_fresh_plans" -m gpu > gpurun_out/r03_s4/pytest_dict.log 2>&1 || { tail -40 gpurun_out/r03_s4/pytest_dict.log; exit 1; }
tail -2 gpurun_out/r03_s4/pytest_dict.log
PQGPU_LIB=$PWD/abx/libdiag.so timeout -k 10 300 python3 -u tools/diag_fused.py 1.5 gpurun_out/r03_s4/diag_c2.json \
  > gpurun_out/r03_s4/diag_c2.txt 2>&1 || { tail -20 gpurun_out/r03_s4/diag_c2.txt; exit 1; }
cat gpurun_out/r03_s4/diag_c2.txt
bash tools/ab_bench.sh r03_s4/tail default abx/libtail10.so abx/libtail25.so
AB_ARGS="--zipf 2.0" bash tools/ab_bench.sh r03_s4/tail_z2 default abx/libtail10.so abx/libtail25.so
