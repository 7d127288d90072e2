#!/bin/bash
# SQ counters per kernel of one C4 column group (diagnostics): bash tools/c4_pmc_group.sh <tag> <group>
set -euo pipefail
TAG=$1; G=$2
OUT=gpurun_out/$TAG/pmc_$G; mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM"; do
  timeout -s KILL 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pass$i" -o run -- \
    python3 bench.py --workload c4 --rows 125000000 --steps 3 --warmup 1 --no-cpu --no-verify --c4-cols $G > "$OUT/pass$i.log" 2>&1 \
    || { tail -20 "$OUT/pass$i.log"; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_kernels.py "$OUT" > "$OUT/summary.txt" || true
cat "$OUT/summary.txt"
