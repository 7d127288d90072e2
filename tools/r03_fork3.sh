#!/bin/bash
# Four-queue launch (strings / other BYTE_ARRAY / fixed-width on queues created with the context):
# tests, then the suite lines in one process (several decoders) without a profiler, C4 125M-row shard.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_fork3}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_binary.py \
  tests/test_gpu_fixtures.py tests/test_gpu_fullsize.py tests/test_c_harness.py tests/test_gpu_parity.py tests/test_dba_carry.py \
  tests/test_gpu_error_epochs.py tests/test_gpu_timeout.py tests/test_gpu_assembly.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 900 python3 tools/bench_suite.py c1_plain_i32 c2_zipf2 c3_mixed c5_levels str_plain str_dict str_dlba str_dba \
  bss_f64 delta_i64 delta_i64_2048 c4_lineitem --cpu-budget 0 > $OUT/suite.jsonl 2> $OUT/suite.err || { tail -30 $OUT/suite.err; exit 1; }
python3 - $OUT/suite.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["workload"], round(d["ms_per_launch"], 3), "ms", round(d.get("hbm_frac", 0), 3))
PY
timeout -k 10 600 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -30 $OUT/bench_c4.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('C4 125M', round(d['ms_per_step'],3), 'ms', round(d['roofline']['frac'],3))" $OUT/bench_c4.json
