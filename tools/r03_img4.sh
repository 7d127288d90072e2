#!/bin/bash
# Unaligned ds_read_b32 in img4: binary / fixture tests (forced one-pass per page too), then A/B against
# the aligned-pair build on the string suite lines.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_img4}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_binary.py \
  tests/test_gpu_fixtures.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
PQGPU_PLAIN_PG=3 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_binary.py \
  > $OUT/pytest_forced.log 2>&1 || { tail -60 $OUT/pytest_forced.log; exit 1; }
tail -1 $OUT/pytest_forced.log
bash tools/ab_suite.sh ${1:-r03_img4}/ab "c3_mixed c4_lineitem str_plain str_dict" default abx/libimg4a.so
