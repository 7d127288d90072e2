#!/bin/bash
# String-path session: BYTE_ARRAY parity tests, then the string suite lines and C4 (125M-row shard)
# under rocprofv3 kernel stats. Each GPU step has its own limit; stop at the first failure.
set -euo pipefail
TAG=${1:-r03_str}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_binary.py \
  tests/test_dba_carry.py tests/test_gpu_fixtures.py tests/test_c_harness.py \
  "tests/test_gpu_fullsize.py::test_c3_full" "tests/test_gpu_fullsize.py::test_c4_lineitem_row_groups" \
  "tests/test_gpu_fullsize.py::test_c4_configured_shard" tests/test_gpu_assembly.py tests/test_assembly_schema.py \
  "tests/test_gpu_fullsize.py::test_c5_full_with_assembly" -m gpu > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
  python3 tools/bench_suite.py c3_mixed c5_levels str_plain str_dict str_dlba str_dba c4_lineitem --cpu-budget 0 \
  > "$OUT/suite.jsonl" 2> "$OUT/suite.err" || { tail -30 "$OUT/suite.err"; exit 1; }
cat "$OUT/suite.jsonl"
python3 tools/kstats.py "$OUT/prof"
timeout -k 10 600 python -u bench.py --workload c4 --rows 125000000 --steps 5 --warmup 2 --no-cpu \
  > "$OUT/bench_c4.json" 2> "$OUT/bench_c4.err" || { tail -30 "$OUT/bench_c4.err"; exit 1; }
cat "$OUT/bench_c4.json"
