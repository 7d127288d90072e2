#!/bin/bash
# Round-3 GPU session: full -m gpu suite, smoke, headline bench, C5 suite line with assembly under
# rocprofv3. Every GPU step has its own time limit; the script stops at the first failure.
set -euo pipefail
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
  || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -30 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5prof" -o run -- \
  python3 tools/bench_suite.py c5_levels --cpu-budget 0 > "$OUT/suite_c5.jsonl" 2> "$OUT/suite_c5.err" \
  || { tail -30 "$OUT/suite_c5.err"; exit 1; }
cat "$OUT/suite_c5.jsonl"
python3 tools/kstats.py "$OUT/c5prof"
