set -e
# C4 column groups alone (125 M rows): the four dictionary-direct string columns, l_comment, and the
# eleven fixed-width columns — each group's launch with the chip to itself, against the whole launch
O=gpurun_out/r06c4s; mkdir -p $O
export TMPDIR=/tmp
for G in "8,9,13,14" "15" "0,1,2,3,4,5,6,7,10,11,12"; do
  timeout -k 10 600 python3 bench.py --workload c4 --rows 125000000 --c4-cols $G --steps 5 --warmup 1 --no-cpu > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c4.json').read().strip().splitlines()[-1])
print('cols $G', round(d['ms_per_step'],3), 'ms', round(d['roofline']['frac'],3))"
done
