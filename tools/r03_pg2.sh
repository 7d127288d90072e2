#!/bin/bash
# k_bin_plain_pg with the short-length candidate filter: forced binary/fixture/parity tests, full-size
# tests, the string suite lines, then C4 at its configured per-GPU shard (125M rows) under rocprofv3.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_pg2}
mkdir -p $OUT
PQGPU_PLAIN_PG=3 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_binary.py tests/test_gpu_fixtures.py tests/test_gpu_parity.py > $OUT/pytest_forced.log 2>&1 || { tail -60 $OUT/pytest_forced.log; exit 1; }
tail -1 $OUT/pytest_forced.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_binary.py \
  > $OUT/pytest_full.log 2>&1 || { tail -60 $OUT/pytest_full.log; exit 1; }
tail -1 $OUT/pytest_full.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 tools/bench_suite.py c3_mixed c4_lineitem str_plain --cpu-budget 0 > $OUT/suite.jsonl 2> $OUT/suite.err || { tail -30 $OUT/suite.err; exit 1; }
cut -c1-200 $OUT/suite.jsonl
python3 tools/seg_kernels.py $OUT/prof/run_kernel_trace.csv --names c3,c4_8M,str_plain > $OUT/per_workload.txt || true
cat $OUT/per_workload.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4prof -o run -- \
  python3 bench.py --workload c4 --rows 125000000 --steps 5 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -30 $OUT/bench_c4.err; exit 1; }
cut -c1-400 $OUT/bench_c4.json
python3 tools/kstats.py $OUT/c4prof | head -20 || true
