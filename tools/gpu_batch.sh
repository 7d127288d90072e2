set -e
O=gpurun_out/r05ab; mkdir -p $O
export TMPDIR=/tmp
bash tools/ab_suite_prof.sh r05ab_s "c3_strings" abx/libprev.so parquet-mr_amd/pqgpu/libpqgpu.so
for L in abx/libprev.so parquet-mr_amd/pqgpu/libpqgpu.so; do
PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 --no-cpu > $O/c4.json 2> $O/c4.err || { tail -30 $O/c4.err; exit 1; }
python3 -c "import json; print('C4 $L', json.load(open('$O/c4.json'))['ms_per_step'])"
done
SUITE="c3_mixed" timeout -k 10 900 python -u tools/bench_suite.py c3_mixed --cpu-budget 0 > $O/c3.jsonl 2> $O/c3.err && cat $O/c3.jsonl | python3 -c "import json,sys; [print(json.loads(l)['workload'], json.loads(l)['ms_per_launch']) for l in sys.stdin]"
PQGPU_LIB=$PWD/abx/libprev.so timeout -k 10 900 python -u tools/bench_suite.py c3_mixed --cpu-budget 0 > $O/c3p.jsonl 2> $O/c3p.err && cat $O/c3p.jsonl | python3 -c "import json,sys; [print('prev', json.loads(l)['workload'], json.loads(l)['ms_per_launch']) for l in sys.stdin]"
