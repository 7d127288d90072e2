set -e
mkdir -p gpurun_out/r05n
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gzip.py tests/test_gpu_binary.py > gpurun_out/r05n/tests.log 2>&1 || { tail -30 gpurun_out/r05n/tests.log; exit 1; }
tail -2 gpurun_out/r05n/tests.log
bash tools/ab_c4prof.sh r05n 8,9,13,14 abx/libbase.so default abx/libnone.so
PQGPU_LIB=$PWD/abx/libdiag.so timeout -k 10 200 python3 tools/diag_lvl.py 0.1 > gpurun_out/r05n/diag_lvl.json
cat gpurun_out/r05n/diag_lvl.json
bash tools/ab_suite_prof.sh r05o "c3_strings" abx/libbase.so parquet-mr_amd/pqgpu/libpqgpu.so
