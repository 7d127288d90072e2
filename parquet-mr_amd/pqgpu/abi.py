"""ctypes mirror of include/pqgpu.h (the C ABI).

Only data layout and constants live here; `native.py` binds the functions of
libpqgpu.so and the oracle binds the same structs for the CPU checker.
"""
import ctypes as C

import numpy as np

ABI_VERSION = 4

# parquet-format Type
BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY = range(8)
TYPE_NAMES = {BOOLEAN: "BOOLEAN", INT32: "INT32", INT64: "INT64", INT96: "INT96", FLOAT: "FLOAT",
              DOUBLE: "DOUBLE", BYTE_ARRAY: "BYTE_ARRAY", FIXED_LEN_BYTE_ARRAY: "FIXED_LEN_BYTE_ARRAY"}

# parquet-format Encoding
PLAIN = 0
PLAIN_DICTIONARY = 2
RLE = 3
BIT_PACKED = 4
DELTA_BINARY_PACKED = 5
DELTA_LENGTH_BYTE_ARRAY = 6
DELTA_BYTE_ARRAY = 7
RLE_DICTIONARY = 8
BYTE_STREAM_SPLIT = 9

# pqg_error
OK = 0
ERR_INVALID_ARG = 1
ERR_UNSUPPORTED = 2
ERR_HIP = 3
ERR_NO_DEVICE = 4
ERR_TIMEOUT = 5
ERR_EOF = 10
ERR_RLE_PAST_END = 11
ERR_BIT_WIDTH = 12
ERR_DICT_ID = 13
ERR_EMPTY_PAGE = 14
ERR_EMPTY_PACKED_RUN = 15
ERR_DELTA_CONFIG = 16
ERR_DELTA_PAST_END = 17
ERR_CORRUPT = 18
ERR_NO_DICTIONARY = 19
ERR_DICT_ENCODING = 20
ERR_CRC = 21

# ColumnMetaData.codec (parquet.thrift CompressionCodec; pqg_codec)
CODEC_UNCOMPRESSED, CODEC_SNAPPY, CODEC_GZIP, CODEC_LZO, CODEC_BROTLI, CODEC_LZ4, CODEC_ZSTD, CODEC_LZ4_RAW = range(8)
COLUMN_DICTIONARY_IDS = 1  # pqg_column_desc.flags: values <- uint32 dictionary ids
PAGE_DBA_CARRY = 1  # pqg_page_desc.flags: DELTA_BYTE_ARRAY page continues the previous page's value (PARQUET-246)
PAGE_NULL_COUNT = 2  # pqg_page_desc.flags: num_nulls holds the V2 header's null count (a verified hint)

ERROR_NAMES = {
    OK: "OK", ERR_INVALID_ARG: "INVALID_ARG", ERR_UNSUPPORTED: "UNSUPPORTED", ERR_HIP: "HIP",
    ERR_NO_DEVICE: "NO_DEVICE", ERR_TIMEOUT: "TIMEOUT", ERR_EOF: "EOF", ERR_RLE_PAST_END: "RLE_PAST_END",
    ERR_BIT_WIDTH: "BIT_WIDTH", ERR_DICT_ID: "DICT_ID", ERR_EMPTY_PAGE: "EMPTY_PAGE",
    ERR_EMPTY_PACKED_RUN: "EMPTY_PACKED_RUN", ERR_DELTA_CONFIG: "DELTA_CONFIG",
    ERR_DELTA_PAST_END: "DELTA_PAST_END", ERR_CORRUPT: "CORRUPT", ERR_NO_DICTIONARY: "NO_DICTIONARY",
    ERR_DICT_ENCODING: "DICT_ENCODING", ERR_CRC: "CRC",
}


class PageDesc(C.Structure):
    """pqg_page_desc (56 bytes)."""
    _fields_ = [
        ("offset", C.c_uint64),
        ("size", C.c_uint32),
        ("num_values", C.c_uint32),
        ("column", C.c_int32),
        ("version", C.c_int32),
        ("encoding", C.c_int32),
        ("rl_encoding", C.c_int32),
        ("dl_encoding", C.c_int32),
        ("rl_byte_length", C.c_uint32),
        ("dl_byte_length", C.c_uint32),
        ("flags", C.c_uint32),
        ("num_nulls", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


PAGE_DTYPE = np.dtype([
    ("offset", "<u8"), ("size", "<u4"), ("num_values", "<u4"), ("column", "<i4"), ("version", "<i4"),
    ("encoding", "<i4"), ("rl_encoding", "<i4"), ("dl_encoding", "<i4"), ("rl_byte_length", "<u4"),
    ("dl_byte_length", "<u4"), ("flags", "<u4"), ("num_nulls", "<u4"), ("reserved", "<u4"),
])
assert PAGE_DTYPE.itemsize == C.sizeof(PageDesc) == 56


class ColumnDesc(C.Structure):
    """pqg_column_desc."""
    _fields_ = [
        ("physical_type", C.c_int32),
        ("type_length", C.c_int32),
        ("max_rep", C.c_int32),
        ("max_def", C.c_int32),
        ("dict_offset", C.c_int64),
        ("dict_size", C.c_uint32),
        ("dict_num_values", C.c_uint32),
        ("dict_encoding", C.c_int32),
        ("flags", C.c_int32),
        ("values", C.c_void_p),
        ("values_capacity", C.c_uint64),
        ("def_levels", C.c_void_p),
        ("rep_levels", C.c_void_p),
        ("levels_capacity", C.c_uint64),
        ("binary_data", C.c_void_p),
        ("binary_capacity", C.c_uint64),
        ("values_written", C.c_uint64),
    ]


class PageHeader(C.Structure):
    """pqg_page_header (parquet.thrift PageHeader fields the reader uses)."""
    _fields_ = [("type", C.c_int32), ("uncompressed_page_size", C.c_int32), ("compressed_page_size", C.c_int32),
                ("has_crc", C.c_int32), ("crc", C.c_uint32), ("num_values", C.c_int32), ("encoding", C.c_int32),
                ("definition_level_encoding", C.c_int32), ("repetition_level_encoding", C.c_int32),
                ("num_nulls", C.c_int32), ("num_rows", C.c_int32), ("definition_levels_byte_length", C.c_int32),
                ("repetition_levels_byte_length", C.c_int32), ("is_compressed", C.c_int32), ("is_sorted", C.c_int32),
                ("reserved", C.c_int32), ("header_offset", C.c_uint64), ("body_offset", C.c_uint64)]


DATA_PAGE, INDEX_PAGE, DICTIONARY_PAGE, DATA_PAGE_V2 = 0, 1, 2, 3


class Status(C.Structure):
    """pqg_status."""
    _fields_ = [
        ("code", C.c_int32),
        ("page", C.c_int32),
        ("value_index", C.c_int64),
        ("message", C.c_char * 240),
    ]

    def as_tuple(self):
        return (int(self.code), int(self.page), int(self.value_index))


class PageError(C.Structure):
    """pqg_page_error (pqg_page_errors: every page's own first error)."""
    _fields_ = [("code", C.c_int32), ("phase", C.c_int32), ("index", C.c_int64)]


# pqg_phase
(PHASE_NONE, PHASE_DICTIONARY, PHASE_RL_INIT, PHASE_DL_INIT, PHASE_DATA_INIT, PHASE_RL_READ, PHASE_DL_READ,
 PHASE_VALUE) = range(8)
LEVELS_REP, LEVELS_DEF = 0, 1  # pqg_levels_kind


class StagedOutput(C.Structure):
    """pqg_staged_output."""
    _fields_ = [("values", C.c_void_p), ("def_levels", C.c_void_p), ("rep_levels", C.c_void_p),
                ("binary", C.c_void_p), ("n_values", C.c_uint64), ("n_slots", C.c_uint64),
                ("n_binary", C.c_uint64)]


# FieldRepetitionType (pqg_repetition)
REQUIRED, OPTIONAL, REPEATED = 0, 1, 2


class SchemaNode(C.Structure):
    """pqg_schema_node."""
    _fields_ = [
        ("parent", C.c_int32),
        ("repetition", C.c_int32),
        ("validity", C.c_void_p),
        ("offsets", C.c_void_p),
        ("capacity", C.c_uint64),
        ("n_entries", C.c_uint64),
    ]


class SchemaLeaf(C.Structure):
    """pqg_schema_leaf."""
    _fields_ = [
        ("node", C.c_int32),
        ("reserved", C.c_int32),
        ("d_def_levels", C.c_void_p),
        ("d_rep_levels", C.c_void_p),
        ("n_slots", C.c_uint64),
    ]


class AssemblyNode(C.Structure):
    """pqg_assembly_node."""
    _fields_ = [
        ("repetition", C.c_int32),
        ("reserved", C.c_int32),
        ("validity", C.c_void_p),
        ("offsets", C.c_void_p),
        ("capacity", C.c_uint64),
        ("n_entries", C.c_uint64),
    ]


def elem_width(physical_type, type_length=0):
    """Width in bytes of one dense output element (pqgpu.h, pqg_column_desc)."""
    return {BOOLEAN: 1, INT32: 4, FLOAT: 4, INT64: 8, DOUBLE: 8, INT96: 12,
            FIXED_LEN_BYTE_ARRAY: type_length, BYTE_ARRAY: 8}[physical_type]


def numpy_dtype(physical_type, type_length=0):
    """numpy dtype of the dense output for a physical type."""
    if physical_type == BOOLEAN:
        return np.dtype(np.uint8)
    if physical_type == INT32:
        return np.dtype("<i4")
    if physical_type == INT64:
        return np.dtype("<i8")
    if physical_type == FLOAT:
        return np.dtype("<f4")
    if physical_type == DOUBLE:
        return np.dtype("<f8")
    if physical_type == BYTE_ARRAY:
        return np.dtype("<i8")  # offsets
    return np.dtype((np.void, elem_width(physical_type, type_length)))

# pqg_ctx_set_dispatch keys (include/pqgpu.h enum pqg_dispatch)
DISPATCH_PLAIN_ONE_PASS = 1
DISPATCH_DICT_DIRECT = 2
DISPATCH_GZIP_PREPASS_MIN = 3  # pqg_gzip_decompress: smallest page (output bytes) for the token pre-pass
DISPATCH_DICT_FUSED = 4  # dictionary pages: 1 = walk + expansion in one launch, 0 = two launches
DISPATCH_NULL_HINTS = 5  # V2 nullable columns: 1 = value kernels from the header null counts (verified), 0 = levels first
