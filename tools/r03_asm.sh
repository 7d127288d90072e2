#!/bin/bash
# Record assembly with 16-byte output stores: assembly / nested tests, A/B on C5.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_asm}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_assembly.py \
  tests/test_gpu_fullsize.py tests/test_c_harness.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab_suite.sh ${1:-r03_asm}/ab "c5_levels" default abx/libasm0.so default abx/libasm0.so
