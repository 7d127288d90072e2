set -e
O=gpurun_out/r06q; mkdir -p $O
export TMPDIR=/tmp
for L in abx/libwalk.so abx/libnu.so parquet-mr_amd/pqgpu/libpqgpu.so abx/libnu.so parquet-mr_amd/pqgpu/libpqgpu.so; do
  NV=""; [ "$L" = abx/libwalk.so ] && NV="--no-verify"
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 tools/bench_suite.py delta_i64 c3_delta --cpu-budget 0 $NV > $O/s.jsonl 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
  python3 -c "
import json
for l in open('$O/s.jsonl'):
    d=json.loads(l); print('$L', d['workload'], round(d['ms_per_launch'],4), round(d.get('hbm_frac', 0) or 0, 3))"
done
