set -e
# BYTE_ARRAY dictionary walks (k_bin_walk over dictionary pages, dictionary entry tiles) launched on the
# plan's stream before the fork (PQG_AB_WALKS_FIRST) instead of first on the BYTE_ARRAY queue, where
# C4's profile showed the 500-wave walk (7 us alone) dispatched late behind the other queues' kernels
# (2.6 ms, delaying the dictionary-direct chain that ends the launch)
O=gpurun_out/r06wf; mkdir -p $O
export TMPDIR=/tmp
PQGPU_LIB=$PWD/abx/libwf.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_binary.py tests/test_gpu_parity.py tests/test_gpu_null_hints.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for L in parquet-mr_amd/pqgpu/libpqgpu.so abx/libwf.so parquet-mr_amd/pqgpu/libpqgpu.so abx/libwf.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 --no-cpu > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c4.json').read().strip().splitlines()[-1])
print('$L', 'c4', round(d['ms_per_step'],3), d['rank0_launch_ms'][:4])"
done
for L in parquet-mr_amd/pqgpu/libpqgpu.so abx/libwf.so; do
  PQGPU_LIB=$PWD/$L timeout -k 10 600 python3 tools/bench_suite.py c3_mixed str_dict str_dict_opt str_dict_16k --cpu-budget 0 > $O/s.jsonl 2> $O/s.err || { tail -20 $O/s.err; exit 1; }
  python3 -c "
import json
for l in open('$O/s.jsonl'):
    d=json.loads(l); print('$L', d['workload'], round(d['ms_per_launch'],4))"
done
