set -e
# Walker segment prefetch (PQG_WALK_PREFETCH: the next LDS segment requested one window ahead) vs HEAD:
# dictionary parity on the variant, then Zipf(2.0) / C2 / str_dict_opt alternating
O=gpurun_out/r06pf; mkdir -p $O
export TMPDIR=/tmp
PQGPU_LIB=$PWD/abx/libpf.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fixtures.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for L in parquet-mr_amd/pqgpu/libpqgpu.so abx/libpf.so parquet-mr_amd/pqgpu/libpqgpu.so abx/libpf.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --zipf 2.0 --no-cpu --no-e2e --steps 20 > $O/z2.json 2> $O/z2.err || { tail -20 $O/z2.err; exit 1; }
  PQGPU_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --no-cpu --no-e2e --steps 20 > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
  python3 -c "
import json
a=json.loads(open('$O/z2.json').read().strip().splitlines()[-1]); b=json.loads(open('$O/c2.json').read().strip().splitlines()[-1])
print('$L', 'zipf2', round(a['ms_per_step'],4), 'c2', round(b['ms_per_step'],4))"
done
