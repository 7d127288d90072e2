#!/bin/bash
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_s7
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_binary.py tests/test_gpu_fixtures.py -m gpu > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
PQGPU_LIB=$PWD/abx/libdiag.so timeout -k 10 300 python3 -u tools/diag_binplain.py str_plain > $OUT/diag_bp.txt 2>&1 || { tail -20 $OUT/diag_bp.txt; exit 1; }
cat $OUT/diag_bp.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 tools/bench_suite.py str_plain c4_lineitem --cpu-budget 0 > $OUT/suite.jsonl 2> $OUT/suite.err || { tail -30 $OUT/suite.err; exit 1; }
cut -c1-200 $OUT/suite.jsonl
python3 tools/seg_kernels.py $OUT/prof/run_kernel_trace.csv --names str_plain,c4_8M || true
