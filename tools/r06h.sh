set -e
O=gpurun_out/r06h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_timeout.py -k "dict or timed" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_binary.py -k "dd or dict or direct" > $O/pytest2.txt 2>&1 || { tail -40 $O/pytest2.txt; exit 1; }
tail -2 $O/pytest2.txt
c2() { # lib dispatch tag
  PQGPU_LIB=$PWD/$1 PQGPU_DISPATCH=$2 timeout -k 10 300 python3 bench.py --steps 30 --warmup 5 --no-cpu --no-e2e > $O/c2.json 2> $O/c2.err || { tail -30 $O/c2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c2.json')); print('C2 $1 [$2]', round(d['ms_per_step'],4), round(d['roofline']['achieved'],1), round(d['roofline']['frac'],3))"
}
for r in 1 2; do
  c2 parquet-mr_amd/pqgpu/libpqgpu.so ""
  c2 parquet-mr_amd/pqgpu/libpqgpu.so "6=0"
  c2 abx/libbase.so ""
done
for a in 1.2 1.5 2; do
  for D in "" "6=0"; do
    PQGPU_DISPATCH=$D timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu --no-e2e --zipf $a > $O/z.json 2> $O/z.err || { tail -30 $O/z.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/z.json')); print('zipf $a [$D]', round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
  done
done
for L in parquet-mr_amd/pqgpu/libpqgpu.so abx/libbase.so parquet-mr_amd/pqgpu/libpqgpu.so abx/libbase.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 tools/bench_suite.py str_dict str_dict_opt str_dict_16k c2_zipf2 --cpu-budget 0 > $O/s.jsonl 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
  python3 -c "
import json
for l in open('$O/s.jsonl'):
    d=json.loads(l); print('$L', d['workload'], round(d['ms_per_launch'],4))"
done
for L in abx/libprio.so abx/libbase.so abx/libprio.so abx/libbase.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 tools/bench_suite.py c3_mixed --cpu-budget 0 > $O/s.jsonl 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/s.jsonl').readline()); print('$L', d['workload'], round(d['ms_per_launch'],4))"
done
for L in parquet-mr_amd/pqgpu/libpqgpu.so abx/libbase.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 --no-cpu --no-e2e > $O/c4.json 2> $O/c4.err || { tail -30 $O/c4.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4.json')); print('$L C4', round(d['ms_per_step'],3), round(d['roofline']['frac'],3))"
done
