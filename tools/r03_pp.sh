#!/bin/bash
# Ping-pong tile buffers in k_bin_plain_pg: binary / fixture / full-size tests (also forced per page),
# string suite lines, C4 125M-row shard.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_pp}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_binary.py \
  tests/test_gpu_fixtures.py tests/test_gpu_fullsize.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
PQGPU_PLAIN_PG=3 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_binary.py \
  tests/test_gpu_fixtures.py > $OUT/pytest_forced.log 2>&1 || { tail -60 $OUT/pytest_forced.log; exit 1; }
tail -1 $OUT/pytest_forced.log
bash tools/ab_suite.sh ${1:-r03_pp}/ab "c3_mixed c4_lineitem str_plain" default
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4prof -o run -- \
  python3 bench.py --workload c4 --rows 125000000 --steps 5 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -30 $OUT/bench_c4.err; exit 1; }
cut -c1-300 $OUT/bench_c4.json
python3 tools/kstats.py $OUT/c4prof | head -4 || true
