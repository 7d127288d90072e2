set -e
# str_plain (20 M PLAIN strings, 1,000 pages: the one-pass tile kernel with its look-back) in two
# processes at once on one GPU, against one process alone, and with one wave per page (1=3, no waits)
O=gpurun_out/r06sh; mkdir -p $O
export TMPDIR=/tmp
run2() {  # $1 tag, $2 dispatch
  PQGPU_DISPATCH=$2 timeout -k 10 240 python3 tools/bench_suite.py str_plain --steps 5 --warmup 1 --cpu-budget 0 > $O/$1_a.jsonl 2> $O/$1_a.err &
  A=$!
  PQGPU_DISPATCH=$2 timeout -k 10 240 python3 tools/bench_suite.py str_plain --steps 5 --warmup 1 --cpu-budget 0 > $O/$1_b.jsonl 2> $O/$1_b.err &
  B=$!
  wait $A; ra=$?; wait $B; rb=$?
  echo "$1 rc $ra $rb"
  [ $ra -eq 0 ] && [ $rb -eq 0 ]
}
timeout -k 10 240 python3 tools/bench_suite.py str_plain --steps 5 --warmup 1 --cpu-budget 0 > $O/solo.jsonl 2> $O/solo.err
run2 pg "1=3"
run2 tiles ""
for f in $O/*.jsonl; do python3 -c "
import json,sys
for l in open('$f'):
    d=json.loads(l); print('$f', round(d['ms_per_launch'],4))"; done
