#!/bin/bash
# Level tiles carried across windows in LDS (no byte stores at window edges): level / optional /
# nested tests, A/B against the previous build on C3 and C5.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_carry}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_assembly.py tests/test_gpu_fixtures.py tests/test_gpu_binary.py tests/test_gpu_fullsize.py tests/test_c_harness.py \
  tests/test_gpu_error_epochs.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
bash tools/ab_suite.sh ${1:-r03_carry}/ab "c3_mixed c5_levels" default abx/libnocarry.so
