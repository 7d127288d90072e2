set -e
# Diagnostic timelines of the fused dictionary kernel (abx/libdiag.so, -DPQG_DIAG) for Zipf 1.5 and 2.0
O=gpurun_out/r06dg; mkdir -p $O
export TMPDIR=/tmp
for z in 1.5 2.0; do
  PQGPU_LIB=$PWD/abx/libdiag.so timeout -k 10 300 python3 tools/diag_fused.py $z $O/diag_z$z.json > $O/diag_z$z.log 2>&1 || { tail -20 $O/diag_z$z.log; exit 1; }
  tail -1 $O/diag_z$z.log | cut -c1-1500
done
