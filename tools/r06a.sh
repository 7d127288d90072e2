set -e
O=gpurun_out/r06a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_null_hints.py tests/test_gpu_binary.py tests/test_gpu_timeout.py tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SUITE="c3_mixed c5_levels delta_i64" bash tools/gpu_round.sh r06a suite
SUITE="c3_mixed" bash tools/gpu_round.sh r06a suiteprof
python3 tools/trace_timeline.py $O/suiteprof > $O/c3_timeline.txt; head -12 $O/c3_timeline.txt; tail -1 $O/c3_timeline.txt
