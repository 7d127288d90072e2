#!/bin/bash
# One-pass PLAIN BYTE_ARRAY kernel on a second queue: tests on multi-column plans, A/B on C3 / C4 (8M and
# the 125M-row shard).
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_fork2}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_binary.py \
  tests/test_gpu_fixtures.py tests/test_gpu_fullsize.py tests/test_c_harness.py tests/test_gpu_parity.py tests/test_dba_carry.py tests/test_gpu_error_epochs.py tests/test_gpu_timeout.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab_suite.sh ${1:-r03_fork2}/ab "c4_lineitem str_dict c3_mixed" default abx/libfork1.so default abx/libfork1.so
for lib in default abx/libfork1.so; do
  n=$(basename $lib .so)
  if [ "$lib" = default ]; then unset PQGPU_LIB; else export PQGPU_LIB=$PWD/$lib; fi
  timeout -k 10 400 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 --no-cpu > $OUT/bench_c4_$n.json 2> $OUT/bench_c4_$n.err || { tail -30 $OUT/bench_c4_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'C4 125M', round(d['ms_per_step'],3), 'ms', round(d['roofline']['frac'],3))" $OUT/bench_c4_$n.json $n
done
