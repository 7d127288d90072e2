#!/bin/bash
# Dictionary-direct BYTE_ARRAY columns (offset scan writes the bytes): tests, A/B against the
# per-value dictionary path (PQGPU_NO_DICT_DIRECT), C4 125M-row shard under rocprofv3.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_dd}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_binary.py \
  tests/test_gpu_fixtures.py tests/test_c_harness.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in dd nodd; do
  if [ $v = nodd ]; then export PQGPU_NO_DICT_DIRECT=1; fi
  timeout -k 10 400 python -u tools/bench_suite.py c4_lineitem str_dict --cpu-budget 0 > $OUT/suite_$v.jsonl 2> $OUT/suite_$v.err || { tail -20 $OUT/suite_$v.err; exit 1; }
  cut -c1-160 $OUT/suite_$v.jsonl
done
unset PQGPU_NO_DICT_DIRECT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c4prof -o run -- \
  python3 bench.py --workload c4 --rows 125000000 --steps 5 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -30 $OUT/bench_c4.err; exit 1; }
cut -c1-300 $OUT/bench_c4.json
python3 tools/kstats.py $OUT/c4prof | head -16 || true
