set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02_a; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 bash tools/ab_bench.sh r02_a/ab default ab/libold.so
timeout -k 10 300 python -u bench.py --gpus 2 --no-cpu --steps 5 > $OUT/bench_g2.json 2> $OUT/bench_g2.err || { tail -30 $OUT/bench_g2.err; exit 1; }
cat $OUT/bench_g2.json
