#!/bin/bash
# Per-page one-pass PLAIN BYTE_ARRAY (k_bin_plain_pg): binary / fixture / parity tests forced through it,
# the full-size C3 / C4 tests, then the string-heavy suite lines per path under rocprofv3.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_pg}
mkdir -p $OUT
PQGPU_PLAIN_PG=3 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_binary.py tests/test_gpu_fixtures.py tests/test_gpu_parity.py > $OUT/pytest_forced.log 2>&1 || { tail -60 $OUT/pytest_forced.log; exit 1; }
tail -2 $OUT/pytest_forced.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py \
  > $OUT/pytest_full.log 2>&1 || { tail -60 $OUT/pytest_full.log; exit 1; }
tail -2 $OUT/pytest_full.log
for mode in 2 0; do
  PQGPU_PLAIN_PG=$mode timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof$mode -o run -- \
    python3 tools/bench_suite.py c3_mixed c4_lineitem --cpu-budget 0 > $OUT/suite$mode.jsonl 2> $OUT/suite$mode.err || { tail -30 $OUT/suite$mode.err; exit 1; }
  cut -c1-220 $OUT/suite$mode.jsonl
  python3 tools/seg_kernels.py $OUT/prof$mode/run_kernel_trace.csv --names c3,c4_8M > $OUT/per_workload$mode.txt || true
  cat $OUT/per_workload$mode.txt
done
