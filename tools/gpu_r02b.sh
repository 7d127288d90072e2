set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02_b; mkdir -p $OUT
timeout -k 10 600 bash tools/ab_bench.sh r02_b/ab default ab/libh1.so ab/libh2.so ab/libh3.so ab/libold.so
AB_ARGS="--zipf 2.0" timeout -k 10 600 bash tools/ab_bench.sh r02_b/ab_z2 default ab/libold.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
