"""pqgpu — MI355X-native Parquet column-page decoder (drop-in for parquet-mr's page-decode path).

Layout:
  abi      ctypes mirror of include/pqgpu.h (the C ABI)
  native   loader of libpqgpu.so (HIP kernels + C ABI); no CPU fallback
  decoder  device-resident batch decode (Decoder, Plan)
  batch    page-batch layout (column chunks, pages, the one-buffer upload tables)
  framing  Thrift page headers -> column chunks
  dist     row-group sharding across GPUs + RCCL gather
"""
from . import abi  # noqa: F401

__all__ = ["abi", "native", "decoder", "batch", "framing", "dist"]
# Page synthesis for tests and benches (the restated parquet-mr writers) is tools/synth/writer.py,
# outside the product package.
