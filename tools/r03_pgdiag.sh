#!/bin/bash
# k_bin_plain_pg: walk-only diagnostic build vs the product on C3 (kernel times under rocprofv3), then SQ
# counters of the product build on C3.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_pgdiag}
mkdir -p $OUT
for lib in default abx/libnoemit.so; do
  n=$(basename $lib .so)
  if [ "$lib" = default ]; then unset PQGPU_LIB; else export PQGPU_LIB=$PWD/$lib; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$n -o run -- \
    python3 tools/bench_suite.py c3_mixed --cpu-budget 0 --no-verify > $OUT/suite_$n.jsonl 2> $OUT/suite_$n.err || { tail -20 $OUT/suite_$n.err; exit 1; }
  python3 tools/kstats.py $OUT/prof_$n | head -4
done
unset PQGPU_LIB
bash tools/r03_pgpmc.sh ${1:-r03_pgdiag}/pmc c3_mixed > /dev/null
grep -A17 "k_bin_plain_pg" $OUT/pmc/summary.txt | head -18
