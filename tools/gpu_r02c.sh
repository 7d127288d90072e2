set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02_c; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 python -u bench.py --workload c4 --rows 125000000 --steps 5 --cpu-budget 10 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { tail -30 $OUT/bench_c4.err; exit 1; }
cat $OUT/bench_c4.json
timeout -k 10 300 python -u bench.py --workload c4 --gpus 2 --rows 8000000 --steps 3 > $OUT/bench_c4_g2.json 2> $OUT/bench_c4_g2.err || { tail -30 $OUT/bench_c4_g2.err; exit 1; }
cat $OUT/bench_c4_g2.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- python3 bench.py --workload c4 --rows 125000000 --steps 5 --no-cpu --no-verify > $OUT/prof_c4.json 2> $OUT/prof_c4.err || { tail -30 $OUT/prof_c4.err; exit 1; }
python3 tools/kstats.py $OUT/prof_c4
timeout -k 10 900 python -u tools/bench_suite.py > $OUT/suite.jsonl 2> $OUT/suite.err || { tail -30 $OUT/suite.err; exit 1; }
cat $OUT/suite.jsonl
