#!/bin/bash
# ZSTD at 10 waves per CU (2 KiB output ring, <= 16 KiB LDS, VGPR target): ZSTD tests on the variant,
# then A/B on the ZSTD suite lines.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_z10}
mkdir -p $OUT
PQGPU_LIB=$PWD/abx/libz10.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_zstd.py > $OUT/pytest_z10.log 2>&1 || { tail -60 $OUT/pytest_z10.log; exit 1; }
tail -1 $OUT/pytest_z10.log
bash tools/ab_suite.sh ${1:-r03_z10}/ab "plain_i64_zstd c2_zstd" default abx/libz10.so
