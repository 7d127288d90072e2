#!/bin/bash
# One GPU-box session: parity tests, bench (with CPU baseline), rocprofv3 kernel stats,
# then separate PMC passes for HBM traffic. Every GPU step has its own time limit and
# the script stops at the first failure (no retries).
# Usage (from the repo root, via gpurun): bash tools/gpu_round.sh <tag> [steps...]
#   steps: tests smoke bench e2e bench2 suite suiteprof prof pmc c4 c4prof wlpmc router diag
#   (default: tests smoke bench prof pmc)
#   env: SUITE="c3_mixed c5_levels" restricts suite / suiteprof / wlpmc to those workloads;
#        TESTS="tests/test_x.py ..." restricts the tests step.
set -euo pipefail
TAG=${1:-run}; shift || true
STEPS=${*:-tests smoke bench prof pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
      tail -3 "$OUT/pytest_gpu.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { tail -30 "$OUT/smoke.log"; exit 1; }
      tail -2 "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
        || { tail -30 "$OUT/bench.err"; exit 1; }
      cat "$OUT/bench.json" ;;
    e2e)
      PQG_HOST_TIMING=1 timeout -k 10 400 python -u bench.py --no-cpu --e2e --steps 5 > "$OUT/bench_e2e.json" 2> "$OUT/bench_e2e.err" \
        || { tail -30 "$OUT/bench_e2e.err"; exit 1; }
      cat "$OUT/bench_e2e.json" ;;
    bench2)
      timeout -k 10 400 python -u bench.py --no-cpu --no-e2e --zipf 2.0 > "$OUT/bench_zipf2.json" 2> "$OUT/bench_zipf2.err" \
        || { tail -30 "$OUT/bench_zipf2.err"; exit 1; }
      cat "$OUT/bench_zipf2.json" ;;
    suite)
      timeout -k 10 900 python -u tools/bench_suite.py ${SUITE:-} --cpu-budget 0 > "$OUT/suite.jsonl" 2> "$OUT/suite.err" \
        || { tail -30 "$OUT/suite.err"; exit 1; }
      python3 - "$OUT/suite.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["workload"], round(d["ms_per_launch"], 4), "ms", round(d.get("hbm_frac", 0), 3))
PY
      ;;
    suiteprof)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/suiteprof" -o run -- \
        python3 tools/bench_suite.py ${SUITE:-} --cpu-budget 0 > "$OUT/suiteprof.jsonl" 2> "$OUT/suiteprof.err" \
        || { tail -30 "$OUT/suiteprof.err"; exit 1; }
      python3 tools/kstats.py "$OUT/suiteprof" ;;
    prof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python3 bench.py --no-cpu --no-e2e > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
        || { tail -30 "$OUT/prof.err"; exit 1; }
      python3 tools/kstats.py "$OUT/prof" ;;
    pmc)
      i=0
      mkdir -p "$OUT/pmc"
      for grp in "FETCH_SIZE" "WRITE_SIZE" \
                 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"; do
        timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc/pass$i" -o run -- \
          python3 bench.py --no-cpu --no-e2e --steps 5 --warmup 1 > "$OUT/pmc/pass$i.log" 2>&1 \
          || { tail -20 "$OUT/pmc/pass$i.log"; exit 1; }
        i=$((i+1))
      done
      python3 tools/pmc_summary.py "$OUT/pmc" --json "$OUT/traffic.json" || true ;;
    c4)
      timeout -k 10 600 python3 bench.py --workload c4 --rows 125000000 --steps 10 --warmup 2 > "$OUT/bench_c4.json" \
        2> "$OUT/bench_c4.err" || { tail -30 "$OUT/bench_c4.err"; exit 1; }
      cat "$OUT/bench_c4.json" ;;
    router)
      timeout -k 10 300 python3 tools/router_latency.py > "$OUT/router_latency.jsonl" 2> "$OUT/router.err" \
        || { tail -20 "$OUT/router.err"; exit 1; }
      cat "$OUT/router_latency.jsonl" ;;
    diag)
      # walk / hand-off / expansion timeline of one C2 launch (diagnostic build abx/libdiag.so)
      PQGPU_LIB=$PWD/abx/libdiag.so timeout -k 10 300 python3 tools/diag_fused.py 1.5 "$OUT/diag_fused.json" \
        > "$OUT/diag_fused.log" 2>&1 || { tail -20 "$OUT/diag_fused.log"; exit 1; }
      tail -30 "$OUT/diag_fused.log" ;;
    c4prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4prof" -o run -- \
        python3 bench.py --workload c4 --rows 125000000 --steps 5 --warmup 1 --no-cpu > "$OUT/c4prof.json" \
        2> "$OUT/c4prof.err" || { tail -30 "$OUT/c4prof.err"; exit 1; }
      python3 tools/kstats.py "$OUT/c4prof" ;;
    wlpmc|strpmc)
      # SQ counters per kernel of the named workloads (separate --pmc passes, 8 SQ each)
      for wl in ${SUITE:-str_plain c3_mixed}; do
        i=0
        mkdir -p "$OUT/strpmc/$wl"
        for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
                   "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM"; do
          timeout -s KILL 400 rocprofv3 --pmc $grp --output-format csv -d "$OUT/strpmc/$wl/pass$i" -o run -- \
            python3 tools/bench_suite.py $wl --steps 3 --warmup 1 --cpu-budget 0 > "$OUT/strpmc/$wl/pass$i.log" 2>&1 \
            || { tail -20 "$OUT/strpmc/$wl/pass$i.log"; exit 1; }
          i=$((i+1))
        done
        python3 tools/pmc_kernels.py "$OUT/strpmc/$wl" > "$OUT/strpmc/$wl/summary.txt" || true
      done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
