#!/bin/bash
# k_levels at 5 waves, dictionary-direct gathers before the offset stores, spin-sleep A/B on C2:
# tests, then the A/B lines, then C4 125M.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_combo}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_assembly.py tests/test_gpu_fixtures.py tests/test_gpu_binary.py tests/test_c_harness.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab_suite.sh ${1:-r03_combo}/lv "c3_mixed c5_levels c4_lineitem" default abx/liblv4.so
bash tools/ab_bench.sh ${1:-r03_combo}/spin default abx/libsl8.so abx/libsl32.so
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4prof -o run -- \
  python3 bench.py --workload c4 --rows 125000000 --steps 5 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -30 $OUT/bench_c4.err; exit 1; }
cut -c1-300 $OUT/bench_c4.json
python3 tools/kstats.py $OUT/c4prof | head -12 || true
