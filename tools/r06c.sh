set -e
O=gpurun_out/r06c; mkdir -p $O
export TMPDIR=/tmp
SUITE="str_dict_16k str_dict_opt" bash tools/gpu_round.sh r06c suiteprof
python3 tools/kstats.py gpurun_out/r06c/suiteprof
