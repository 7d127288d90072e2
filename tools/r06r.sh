set -e
O=gpurun_out/r06r; mkdir -p $O
export TMPDIR=/tmp
PQGPU_LIB=$PWD/abx/libl8.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "delta or DELTA or optional" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for L in abx/libl8.so parquet-mr_amd/pqgpu/libpqgpu.so abx/libl8.so parquet-mr_amd/pqgpu/libpqgpu.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 tools/bench_suite.py delta_i64 c3_delta c3_mixed --cpu-budget 0 > $O/s.jsonl 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
  python3 -c "
import json
for l in open('$O/s.jsonl'):
    d=json.loads(l); print('$L', d['workload'], round(d['ms_per_launch'],4), round(d.get('hbm_frac', 0) or 0, 3))"
done
for L in abx/libl8.so parquet-mr_amd/pqgpu/libpqgpu.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 --no-cpu --no-e2e > $O/c4.json 2> $O/c4.err || { tail -30 $O/c4.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4.json')); print('$L C4', round(d['ms_per_step'],3), round(d['roofline']['frac'],3))"
done
