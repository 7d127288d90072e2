#!/bin/bash
# Collect rocprofv3 PMC counters for the bench's dominant kernel, one pass per group
# (separate --pmc passes, kernel-trace only; see MI355X_MICROARCH.md §rocprofv3).
# Usage: tools/pmc.sh <outdir> [bench args...]
set -e
OUT=$1; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pass$i" -o run -- python3 bench.py --no-cpu "$@" > "$OUT/pass$i.log" 2>&1
  i=$((i+1))
done
