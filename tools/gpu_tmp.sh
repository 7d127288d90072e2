set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r02_bin; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "binary or fixture or fullsize or harness" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for lib in default ab/libbase.so ab/libbw1k.so ab/libnostage.so; do
  if [ $lib = default ]; then unset PQGPU_LIB; else export PQGPU_LIB=$PWD/$lib; fi
  timeout -k 10 600 python -u tools/bench_suite.py str_plain str_dict str_dlba c3_mixed c4_lineitem --cpu-budget 0 --steps 10 > $OUT/suite_$(basename $lib .so).jsonl 2>/dev/null || exit 1
  python3 -c "
import json,sys
for l in open(sys.argv[1]):
    d=json.loads(l); print(sys.argv[2], d['workload'], round(d['ms_per_launch'],3), 'ms', round(d['hbm_frac'],3))
" $OUT/suite_$(basename $lib .so).jsonl $lib
done
