#!/bin/bash
# Dictionary-direct with the LDS sized per launch (dictionaries up to 24 KiB): tests, A/B against the
# previous build on C4 8M / str_dict, C4 125M-row shard.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_dd2}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_binary.py \
  tests/test_gpu_fixtures.py tests/test_gpu_fullsize.py tests/test_c_harness.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab_suite.sh ${1:-r03_dd2}/ab "c4_lineitem str_dict" default abx/libprev.so default abx/libprev.so
timeout -k 10 600 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -30 $OUT/bench_c4.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('C4 125M', round(d['ms_per_step'],3), 'ms', round(d['roofline']['frac'],3))" $OUT/bench_c4.json
