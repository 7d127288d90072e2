set -e
# lane_rows_to_tiles for BSS doubles, k_bin_offsets, k_dd_str / k_dd_gstr offsets: parity, then A/B vs HEAD
O=gpurun_out/r06y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_binary.py tests/test_gpu_parity.py tests/test_gpu_fixtures.py tests/test_dba_carry.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for L in abx/libhead.so parquet-mr_amd/pqgpu/libpqgpu.so abx/libhead.so parquet-mr_amd/pqgpu/libpqgpu.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 tools/bench_suite.py bss_f64 str_plain str_dict str_dict_opt str_dict_16k str_dlba delta_i64 --cpu-budget 0 > $O/s.jsonl 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
  python3 -c "
import json
for l in open('$O/s.jsonl'):
    d=json.loads(l); print('$L', d['workload'], round(d['ms_per_launch'],4), round(d.get('hbm_frac', 0) or 0, 3))"
done
for L in abx/libhead.so parquet-mr_amd/pqgpu/libpqgpu.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 tools/bench_suite.py c4_lineitem --cpu-budget 0 > $O/c4.jsonl 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
  python3 -c "
import json
for l in open('$O/c4.jsonl'):
    d=json.loads(l); print('$L', d['workload'], round(d['ms_per_launch'],4), round(d.get('hbm_frac', 0) or 0, 3))"
done
