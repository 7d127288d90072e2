set -e
mkdir -p gpurun_out/r05c
for g in 0,1,2 10,11,12 4,5,6,7 3 8,9,13,14 15; do
  timeout -k 10 300 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 --no-cpu --c4-cols $g > gpurun_out/r05c/c4_$g.json 2> gpurun_out/r05c/c4_$g.err
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r05c/c4_$g.json')); print('$g', round(d['ms_per_step'],3), 'ms', round(d['roofline']['frac'],3), round(d['roofline']['algorithmic_bytes_per_launch']/1e9,2),'GB')"
done
