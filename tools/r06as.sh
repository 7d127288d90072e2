set -e
# k_asm_onepass<MD>: depth-sized registers, 32-bit offsets image, one look-back loop for all depths — parity, A/B
O=gpurun_out/r06as; mkdir -p $O
export TMPDIR=/tmp
PQGPU_LIB=$PWD/abx/libasm16k.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_assembly.py tests/test_gpu_fullsize.py -k "assembl or c5 or nested or record" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for L in abx/libasm8k.so abx/libasm16k.so abx/libasm8k.so abx/libasm16k.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 tools/bench_suite.py c5_levels --cpu-budget 0 > $O/s.jsonl 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
  python3 -c "
import json
for l in open('$O/s.jsonl'):
    d=json.loads(l); a=d.get('assembly') or {}; print('$L', d['workload'], round(d['ms_per_launch'],4), round(d.get('hbm_frac', 0) or 0, 3), 'asm_ms', round(a.get('assembly_ms', 0),4))"
done
