set -e
O=gpurun_out/r06b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_binary.py -k "dictionary_direct or short_buffer" tests/test_gpu_fixtures.py tests/test_gpu_null_hints.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SUITE="str_dict str_dict_opt str_dict_16k c3_mixed" bash tools/gpu_round.sh r06b suite
PQGPU_DISPATCH=5=0 SUITE="c3_mixed" bash tools/gpu_round.sh r06b_nohint suite
bash tools/gpu_round.sh r06b bench
