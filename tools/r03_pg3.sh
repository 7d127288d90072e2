#!/bin/bash
# Dictionary-string scatter copy, fast tile guess, k_bin_plain_pg at 5 waves: tests, A/B of the
# occupancy variants on the string suite lines, C4 125M-row shard under rocprofv3.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_pg3}
mkdir -p $OUT
PQGPU_PLAIN_PG=3 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_binary.py tests/test_gpu_fixtures.py tests/test_gpu_parity.py > $OUT/pytest_forced.log 2>&1 || { tail -60 $OUT/pytest_forced.log; exit 1; }
tail -1 $OUT/pytest_forced.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_binary.py \
  tests/test_gpu_fixtures.py tests/test_c_harness.py > $OUT/pytest_full.log 2>&1 || { tail -60 $OUT/pytest_full.log; exit 1; }
tail -1 $OUT/pytest_full.log
bash tools/ab_suite.sh ${1:-r03_pg3}/ab "c3_mixed c4_lineitem str_plain str_dict" default abx/libpg6.so abx/libbp5.so
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4prof -o run -- \
  python3 bench.py --workload c4 --rows 125000000 --steps 5 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -30 $OUT/bench_c4.err; exit 1; }
cut -c1-300 $OUT/bench_c4.json
python3 tools/kstats.py $OUT/c4prof | head -16 || true
