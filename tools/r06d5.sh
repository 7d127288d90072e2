set -e
# k_delta at 5 waves per SIMD for 8-byte values too (96 VGPRs, 108 B scratch) vs HEAD (122 VGPRs, 4 waves)
O=gpurun_out/r06d5; mkdir -p $O
export TMPDIR=/tmp
PQGPU_LIB=$PWD/abx/libd5.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "delta or DELTA" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for L in parquet-mr_amd/pqgpu/libpqgpu.so abx/libd5.so parquet-mr_amd/pqgpu/libpqgpu.so abx/libd5.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 tools/bench_suite.py delta_i64 delta_i64_2048 c3_delta --cpu-budget 0 > $O/s.jsonl 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
  python3 -c "
import json
for l in open('$O/s.jsonl'):
    d=json.loads(l); print('$L', d['workload'], round(d['ms_per_launch'],4), round(d.get('hbm_frac', 0) or 0, 3))"
done
