set -e
# Diagnostic: k_levels on C3 (levels first: PQGPU_DISPATCH=5=0) with and without the width-1 expansion
# (abx/liblvnoexp.so: counts only, no level written; --no-verify)
O=gpurun_out/r06lv; mkdir -p $O
export TMPDIR=/tmp
for L in parquet-mr_amd/pqgpu/libpqgpu.so abx/liblvnoexp.so; do
  n=$(basename $L .so)
  PQGPU_DISPATCH=5=0 PQGPU_LIB=$PWD/$L timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- \
    python3 tools/bench_suite.py c3_mixed --cpu-budget 0 --no-verify --steps 5 --warmup 1 > $O/$n.jsonl 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 tools/kstats.py $O/$n | grep -i "levels\|scan_off"
done
