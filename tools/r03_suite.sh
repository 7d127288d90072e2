#!/bin/bash
# The suite (every workload line) under rocprofv3 kernel stats, per-workload kernel medians, then the
# C4 125M-row shard.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_suite}
mkdir -p $OUT
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
  python3 tools/bench_suite.py c1_plain_i32 c2_zipf2 c3_mixed c5_levels str_plain str_dict str_dlba str_dba bss_f64 delta_i64 \
  delta_i64_2048 c4_lineitem plain_i64_zstd --cpu-budget 0 > $OUT/suite.jsonl 2> $OUT/suite.err || { tail -30 $OUT/suite.err; exit 1; }
python3 - $OUT/suite.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["workload"], round(d["ms_per_launch"], 3), "ms", round(d.get("hbm_frac", 0), 3))
PY
python3 tools/seg_kernels.py $OUT/prof/run_kernel_trace.csv --names c1,c2_zipf2,c3,c5,str_plain,str_dict,str_dlba,str_dba,bss,delta_i64,delta_2048,c4_8M,zstd > $OUT/per_workload.txt || true
timeout -k 10 600 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -30 $OUT/bench_c4.err; exit 1; }
cut -c1-200 $OUT/bench_c4.json
