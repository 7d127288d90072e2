#!/bin/bash
# Session: one-pass PLAIN BYTE_ARRAY path (k_bin_bases + k_bin_plain) parity, then the string suite.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03_s5
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_binary.py \
  tests/test_gpu_fixtures.py tests/test_c_harness.py tests/test_dba_carry.py \
  "tests/test_gpu_fullsize.py::test_c3_full" "tests/test_gpu_fullsize.py::test_c4_lineitem_row_groups" \
  "tests/test_gpu_fullsize.py::test_c4_configured_shard" -m gpu > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 tools/bench_suite.py c3_mixed str_plain str_dict c4_lineitem --cpu-budget 0 \
  > $OUT/suite.jsonl 2> $OUT/suite.err || { tail -30 $OUT/suite.err; exit 1; }
cut -c1-220 $OUT/suite.jsonl
python3 tools/seg_kernels.py $OUT/prof/run_kernel_trace.csv --names c3,str_plain,str_dict,c4_8M || true
timeout -k 10 600 python -u bench.py --workload c4 --rows 125000000 --steps 5 --warmup 2 --no-cpu \
  > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -30 $OUT/bench_c4.err; exit 1; }
cut -c1-300 $OUT/bench_c4.json
