set -e
O=gpurun_out/r06s; mkdir -p $O
export TMPDIR=/tmp
SUITE="delta_i64" bash tools/gpu_round.sh r06s wlpmc
