#!/bin/bash
# k_levels at 5 waves per SIMD (slimmer LDS): level / optional-column tests, A/B against 4 waves.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_lv}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_assembly.py tests/test_gpu_fixtures.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab_suite.sh ${1:-r03_lv}/ab "c3_mixed c5_levels" default abx/liblv4.so
