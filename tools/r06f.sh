set -e
O=gpurun_out/r06f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SUITE="str_dict_16k str_dict_opt str_dict" bash tools/gpu_round.sh r06f suite
SUITE="c3_mixed c5_levels delta_i64" bash tools/gpu_round.sh r06f wlpmc
