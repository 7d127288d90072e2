set -e
# Scalar packed-run threshold of the dictionary walk (32 product / 16 / 8 data bytes): fused C2 and Zipf(2.0)
O=gpurun_out/r06pk; mkdir -p $O
export TMPDIR=/tmp
for z in 2.0 1.5; do
for L in parquet-mr_amd/pqgpu/libpqgpu.so abx/libpk16.so abx/libpk8.so parquet-mr_amd/pqgpu/libpqgpu.so abx/libpk16.so abx/libpk8.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu --no-e2e --zipf $z > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$L zipf $z', round(d['ms_per_step'],4), round(d['roofline']['frac'],3))"
done
done
