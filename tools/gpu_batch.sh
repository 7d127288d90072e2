set -e
O=gpurun_out/r05u; mkdir -p $O
PQG_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --no-cpu --e2e --steps 5 > $O/e2e.json 2> $O/e2e.err || { tail -30 $O/e2e.err; exit 1; }
grep pqg_decode_host $O/e2e.err | tail -6
PQGPU_LIB=$PWD/abx/libt16.so PQG_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --no-cpu --e2e --steps 5 > $O/e2e16.json 2> $O/e2e16.err || { tail -30 $O/e2e16.err; exit 1; }
grep pqg_decode_host $O/e2e16.err | tail -6
python3 -c "
import json
for f in ['$O/e2e.json','$O/e2e16.json']:
    d=json.load(open(f))['e2e_host_path']; print(f, round(d['output_gb_per_s'],1), round(d['frac_of_d2h_ceiling'],3), round(d['link']['d2h_pinned_gbs'],1))"
timeout -k 10 600 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 --no-cpu --dict-split > $O/c4_split.json 2> $O/c4_split.err || { tail -30 $O/c4_split.err; exit 1; }
timeout -k 10 600 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 --no-cpu > $O/c4.json 2> $O/c4.err || { tail -30 $O/c4.err; exit 1; }
python3 -c "
import json
for f in ['$O/c4_split.json','$O/c4.json']:
    d=json.load(open(f)); print(f, d['ms_per_step'])"
