set -e
# Diagnostic: DELTA steps stored with a transposed (1 KiB per instruction) pattern, values wrong (--no-verify)
O=gpurun_out/r06v; mkdir -p $O
export TMPDIR=/tmp
for L in parquet-mr_amd/pqgpu/libpqgpu.so abx/libtst.so parquet-mr_amd/pqgpu/libpqgpu.so abx/libtst.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 tools/bench_suite.py delta_i64 delta_i64_2048 c3_delta --cpu-budget 0 --no-verify > $O/s.jsonl 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
  python3 -c "
import json
for l in open('$O/s.jsonl'):
    d=json.loads(l); print('$L', d['workload'], round(d['ms_per_launch'],4), round(d.get('hbm_frac', 0) or 0, 3))"
done
