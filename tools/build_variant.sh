#!/bin/bash
# Diagnostic build of libpqgpu.so with extra defines (A/B experiments; loaded through PQGPU_LIB):
#   bash tools/build_variant.sh abx/libnoval.so -DPQG_XT_NOVALUE
set -euo pipefail
OUT=$1; shift
C=parquet-mr_amd/csrc
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -shared "$@" -o "$OUT" \
  $C/pqgpu_kernels.hip $C/pqgpu_binary.hip $C/pqgpu_assembly.hip $C/pqgpu_snappy.hip $C/pqgpu_zstd.hip $C/pqgpu_lz4.hip $C/pqgpu_gzip.hip \
  $C/pqgpu_api.hip $C/pqgpu_framing.cpp $C/pqgpu_reader.cpp -Wl,--no-undefined
