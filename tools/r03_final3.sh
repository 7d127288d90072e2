#!/bin/bash
# Final tree: every GPU test, smoke, the C2 bench, then the dictionary-direct A/B and the C4 shard.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_final3}
mkdir -p $OUT
bash tools/gpu_round.sh ${1:-r03_final3} tests smoke bench
bash tools/ab_suite.sh ${1:-r03_final3}/ab "c4_lineitem str_dict" default abx/libprev.so
timeout -k 10 600 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -30 $OUT/bench_c4.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('C4 125M', round(d['ms_per_step'],3), 'ms', round(d['roofline']['frac'],3))" $OUT/bench_c4.json
