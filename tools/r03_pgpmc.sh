#!/bin/bash
# SQ counters per kernel of C3 (k_bin_plain_pg) in separate --pmc passes (8 SQ counters each).
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_pgpmc}
WL=${2:-c3_mixed}
mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM"; do
  timeout -s KILL 400 rocprofv3 --pmc $grp --output-format csv -d $OUT/pass$i -o run -- \
    python3 tools/bench_suite.py $WL --steps 3 --warmup 1 --cpu-budget 0 > $OUT/pass$i.log 2>&1 || { tail -20 $OUT/pass$i.log; exit 1; }
  i=$((i+1))
done
python3 tools/pmc_kernels.py $OUT > $OUT/summary.txt || true
cat $OUT/summary.txt
