"""ctypes binding of libpqgpu.so (the C ABI in include/pqgpu.h).

The HIP library is the only decode path: if it is missing or has no device,
the calls below raise — there is no CPU fallback in the product.
"""
import ctypes as C
import os

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
# PQGPU_LIB selects a diagnostic build (tools/); the product is libpqgpu.so
LIB_PATH = os.environ.get("PQGPU_LIB") or os.path.join(_HERE, "libpqgpu.so")
_LIB = None

EXPORTS = [
    "pqg_abi_version", "pqg_device_count", "pqg_ctx_create", "pqg_ctx_destroy", "pqg_ctx_stream", "pqg_ctx_set_dispatch",
    "pqg_decode",
    "pqg_sync", "pqg_plan_create", "pqg_plan_launch", "pqg_plan_kernel_count", "pqg_plan_timeout_fallbacks", "pqg_plan_plain_fallbacks",
    "pqg_plan_null_hint_fallbacks",
    "pqg_plan_destroy",
    "pqg_decode_host", "pqg_unpack_runs", "pqg_router_read", "pqg_router_read_runs", "pqg_router_read_page",
    "pqg_router_cache_lookup", "pqg_router_cache_stats", "pqg_error_name",
    "pqg_page_errors", "pqg_plan_page_errors", "pqg_host_input", "pqg_decode_staged", "pqg_staged_column",
    "pqg_copy_out", "pqg_assemble", "pqg_assemble_schema",
    "pqg_snappy_decompress", "pqg_snappy_sync", "pqg_zstd_decompress", "pqg_zstd_sync",
    "pqg_lz4_raw_decompress", "pqg_lz4_raw_sync", "pqg_gzip_decompress", "pqg_gzip_sync", "pqg_crc32", "pqg_frame_chunk", "pqg_pages_from_headers",
    # include/pqgpu_reader.h (the ValuesReader contract over a decoded batch)
    "pqg_vr_init_from_page", "pqg_vr_remaining", "pqg_vr_read_dictionary_id", "pqg_vr_read_boolean",
    "pqg_vr_read_integer", "pqg_vr_read_long", "pqg_vr_read_float", "pqg_vr_read_double", "pqg_vr_read_bytes",
    "pqg_vr_skip", "pqg_vr_skip_n", "pqg_lr_init_from_page", "pqg_lr_remaining", "pqg_lr_read_integer",
    "pqg_lr_skip", "pqg_java_exception",
]


class PqgError(RuntimeError):
    """A decode error; mirrors org.apache.parquet.io.ParquetDecodingException."""

    def __init__(self, code, status=None, what=""):
        self.code = int(code)
        self.status = status
        name = abi.ERROR_NAMES.get(self.code, str(self.code))
        msg = f"{what}: {name}" if what else name
        if status is not None:
            msg += f" (page {status.page}, index {status.value_index}): {status.message.decode(errors='replace')}"
        super().__init__(msg)


def lib():
    """Load libpqgpu.so; raises if the HIP extension was not built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"HIP extension missing: {LIB_PATH} (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        vp, i32, u64 = C.c_void_p, C.c_int, C.c_uint64
        L.pqg_abi_version.restype = i32
        L.pqg_device_count.restype = i32
        L.pqg_ctx_create.argtypes = [i32, vp, C.POINTER(vp)]
        L.pqg_ctx_destroy.argtypes = [vp]
        L.pqg_ctx_stream.argtypes = [vp]
        L.pqg_ctx_stream.restype = vp
        L.pqg_ctx_set_dispatch.argtypes = [vp, i32, i32]
        L.pqg_decode.argtypes = [vp, vp, u64, vp, i32, vp, i32, vp, C.POINTER(abi.Status)]
        L.pqg_sync.argtypes = [vp, C.POINTER(abi.Status)]
        L.pqg_plan_create.argtypes = [vp, vp, u64, vp, i32, vp, i32, C.POINTER(vp), C.POINTER(abi.Status)]
        L.pqg_plan_launch.argtypes = [vp]
        L.pqg_plan_kernel_count.argtypes = [vp]
        L.pqg_plan_timeout_fallbacks.argtypes = [vp]
        L.pqg_plan_plain_fallbacks.argtypes = [vp]
        L.pqg_plan_null_hint_fallbacks.argtypes = [vp]
        L.pqg_plan_destroy.argtypes = [vp]
        L.pqg_decode_host.argtypes = [vp, vp, u64, vp, i32, vp, i32, vp, C.POINTER(abi.Status)]
        L.pqg_unpack_runs.argtypes = [vp, i32, vp, vp, vp, vp, vp, i32]
        L.pqg_router_read.argtypes = [vp, i32, vp, C.c_size_t, i32, vp]
        L.pqg_router_read_runs.argtypes = [vp, i32, vp, C.c_size_t, vp, vp, i32, vp]
        L.pqg_router_read_page.argtypes = [vp, i32, vp, C.c_size_t, i32, vp]
        L.pqg_router_cache_lookup.argtypes = [vp, i32, vp, C.c_size_t, i32, vp, C.POINTER(i32)]
        L.pqg_router_cache_stats.argtypes = [vp, C.POINTER(u64), C.POINTER(u64)]
        L.pqg_page_errors.argtypes = [vp, vp, i32]
        L.pqg_plan_page_errors.argtypes = [vp, vp, i32]
        L.pqg_host_input.argtypes = [vp, u64, C.POINTER(vp)]
        L.pqg_decode_staged.argtypes = [vp, u64, vp, i32, vp, i32, vp, C.POINTER(abi.Status)]
        L.pqg_staged_column.argtypes = [vp, i32, C.POINTER(abi.StagedOutput)]
        L.pqg_copy_out.argtypes = [vp, vp, u64]
        L.pqg_copy_out.restype = None
        L.pqg_assemble.argtypes = [vp, vp, vp, u64, vp, i32, C.POINTER(u64), C.POINTER(abi.Status)]
        L.pqg_assemble_schema.argtypes = [vp, vp, i32, vp, i32, C.POINTER(u64), C.POINTER(abi.Status)]
        L.pqg_snappy_decompress.argtypes = [vp, vp, u64, vp, u64, vp, i32, vp]
        L.pqg_snappy_sync.argtypes = [vp, vp, i32, C.POINTER(abi.Status)]
        L.pqg_zstd_decompress.argtypes = [vp, vp, u64, vp, u64, vp, i32, vp]
        L.pqg_zstd_sync.argtypes = [vp, vp, i32, C.POINTER(abi.Status)]
        L.pqg_lz4_raw_decompress.argtypes = [vp, vp, u64, vp, u64, vp, i32, vp]
        L.pqg_lz4_raw_sync.argtypes = [vp, vp, i32, C.POINTER(abi.Status)]
        L.pqg_gzip_decompress.argtypes = [vp, vp, u64, vp, u64, vp, i32, vp]
        L.pqg_gzip_sync.argtypes = [vp, vp, i32, C.POINTER(abi.Status)]
        L.pqg_crc32.argtypes = [C.c_uint32, vp, u64]
        L.pqg_crc32.restype = C.c_uint32
        L.pqg_frame_chunk.argtypes = [vp, u64, C.c_int64, i32, vp, i32, C.POINTER(i32), C.POINTER(abi.Status)]
        L.pqg_pages_from_headers.argtypes = [vp, i32, i32, u64, i32, vp, vp, i32, C.POINTER(i32), C.POINTER(abi.Status)]
        L.pqg_error_name.argtypes = [i32]
        L.pqg_error_name.restype = C.c_char_p
        if L.pqg_abi_version() != abi.ABI_VERSION:
            raise RuntimeError("libpqgpu.so ABI version mismatch")
        _LIB = L
    return _LIB


def check(rc, status=None, what=""):
    if rc != abi.OK:
        raise PqgError(rc, status, what)
