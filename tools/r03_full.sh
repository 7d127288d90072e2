#!/bin/bash
# Full GPU test run + the string / codec suite lines under rocprofv3 kernel stats.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_full}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 tools/bench_suite.py c3_mixed str_plain str_dict c4_lineitem plain_i64_zstd --cpu-budget 0 \
  > $OUT/suite.jsonl 2> $OUT/suite.err || { tail -30 $OUT/suite.err; exit 1; }
cut -c1-200 $OUT/suite.jsonl
python3 tools/seg_kernels.py $OUT/prof/run_kernel_trace.csv --names c3,str_plain,str_dict,c4_8M,zstd || true
