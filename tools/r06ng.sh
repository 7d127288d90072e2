set -e
# DELTA_LENGTH lengths (NEG) through the segment expansion: parity (incl. negative lengths), then A/B vs HEAD
O=gpurun_out/r06ng; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_binary.py tests/test_gpu_parity.py -k "dlba or DLBA or delta or DELTA or binary_errors or dba or DBA" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for L in abx/libhead.so parquet-mr_amd/pqgpu/libpqgpu.so abx/libhead.so parquet-mr_amd/pqgpu/libpqgpu.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 tools/bench_suite.py str_dlba delta_i64 --cpu-budget 0 > $O/s.jsonl 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
  python3 -c "
import json
for l in open('$O/s.jsonl'):
    d=json.loads(l); print('$L', d['workload'], round(d['ms_per_launch'],4), round(d.get('hbm_frac', 0) or 0, 3))"
done
