set -e
O=gpurun_out/r06l; mkdir -p $O
export TMPDIR=/tmp
SUITE="str_dict_opt" bash tools/gpu_round.sh r06l suiteprof
python3 tools/trace_timeline.py $O/suiteprof 50 > $O/opt_timeline.txt; cat $O/opt_timeline.txt
