set -e
O=gpurun_out/r05v; mkdir -p $O
export TMPDIR=/tmp
PQG_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --no-cpu --e2e --steps 5 > $O/e2e.json 2> $O/e2e.err || { tail -30 $O/e2e.err; exit 1; }
python3 -c "
import json
d=json.load(open('$O/e2e.json'))['e2e_host_path']
print(json.dumps({k:v for k,v in d.items() if k not in ('path','native_call_s','with_python_alloc_s')}))"
for m in 1 2; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pm$m -o run -- python3 bench.py --workload c4 --rows 125000000 --steps 5 --warmup 1 --no-cpu --no-verify --c4-cols 15 --plain-mode $m > $O/pm$m.json 2> $O/pm$m.err || { tail -20 $O/pm$m.err; exit 1; }
echo "== plain mode $m"; python3 tools/kstats.py $O/pm$m | head -6
done
for m in 1 2; do
timeout -k 10 600 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 --no-cpu --plain-mode $m > $O/c4_pm$m.json 2> $O/c4_pm$m.err || { tail -30 $O/c4_pm$m.err; exit 1; }
python3 -c "import json; print('C4 plain mode $m', json.load(open('$O/c4_pm$m.json'))['ms_per_step'])"
done
