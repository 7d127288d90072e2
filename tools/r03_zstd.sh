#!/bin/bash
# ZSTD session: the ZSTD parity tests, then the codec suite lines under rocprofv3 kernel stats.
set -euo pipefail
TAG=${1:-r03_zstd}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_zstd.py \
  tests/test_gpu_snappy.py -m gpu > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 tools/bench_suite.py plain_i64_zstd c2_zstd --cpu-budget 0 --steps 5 \
  > "$OUT/suite.jsonl" 2> "$OUT/suite.err" || { tail -30 "$OUT/suite.err"; exit 1; }
cat "$OUT/suite.jsonl"
python3 tools/kstats.py "$OUT/prof"
