set -e
# EXPERIMENT: every dictionary run header on the scalar path (abx/libser.so) vs the window walk: fused C2 / Zipf(2.0)
O=gpurun_out/r06ser; mkdir -p $O
export TMPDIR=/tmp
PQGPU_LIB=$PWD/abx/libser.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "dict or DICT or zipf or c2" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for z in 2.0 1.5; do
for L in parquet-mr_amd/pqgpu/libpqgpu.so abx/libser.so parquet-mr_amd/pqgpu/libpqgpu.so abx/libser.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --zipf $z > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$L zipf $z', round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
done
done
