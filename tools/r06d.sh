set -e
O=gpurun_out/r06d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_binary.py tests/test_gpu_timeout.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SUITE="str_dict str_dict_opt str_dict_16k c2_zipf2" bash tools/gpu_round.sh r06d suite
SUITE="str_dict_16k" bash tools/gpu_round.sh r06d suiteprof
for L in abx/libnohop.so parquet-mr_amd/pqgpu/libpqgpu.so abx/libnohop.so parquet-mr_amd/pqgpu/libpqgpu.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --no-cpu --no-e2e > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b.json')); print('$L', round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
  PQGPU_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --zipf 2.0 > $O/b2.json 2> $O/b2.err || { tail -20 $O/b2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b2.json')); print('$L zipf2', round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
done
