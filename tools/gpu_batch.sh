set -e
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_hybrid_sections.py tests/test_gpu_fixtures.py tests/test_gpu_fullsize.py tests/test_gpu_assembly.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_suite_prof.sh r05s_lv "c3_mixed c5_levels" abx/libbase.so parquet-mr_amd/pqgpu/libpqgpu.so
bash tools/c4_pmc_group.sh r05s 8,9,13,14
