"""Page framing: Thrift-compact PageHeader parsing and column-chunk page splitting.

Restates what parquet-mr's ParquetFileReader.Chunk.readAllPages does for one
column chunk (parquet-hadoop/.../ParquetFileReader.java:1824-1979) with the
header read by Util.readPageHeader (parquet-format-structures/.../Util.java:127-131,
Thrift TCompactProtocol). Chunks are UNCOMPRESSED, SNAPPY, GZIP, ZSTD or LZ4_RAW (ColumnMetaData.codec):
compressed pages keep their compressed bodies (codec / uncompressed_size on the Page) and are
decompressed on the GPU by Decoder.upload_chunks (pqg_snappy / zstd / lz4_raw / gzip_decompress).
The C-ABI form of the same walk is pqg_frame_chunk (frame_chunk_native below). The result is a
batch.ColumnChunk whose pages feed batch.build_batch -> the device decoder.

This is host-side metadata handling (headers, offsets); no page data is decoded
here.
"""
import struct

from . import abi
from .batch import ColumnChunk, Page

# PageType (parquet.thrift)
DATA_PAGE, INDEX_PAGE, DICTIONARY_PAGE, DATA_PAGE_V2 = 0, 1, 2, 3

# TCompactProtocol types
T_STOP, T_TRUE, T_FALSE, T_BYTE, T_I16, T_I32, T_I64, T_DOUBLE, T_BINARY, T_LIST, T_SET, T_MAP, T_STRUCT = range(13)


class ThriftError(ValueError):
    pass


class _Reader:
    def __init__(self, buf, pos):
        self.buf = buf if isinstance(buf, (bytes, bytearray, memoryview)) else memoryview(buf).cast("B")
        self.pos = pos

    def byte(self):
        if self.pos >= len(self.buf):
            raise ThriftError("truncated thrift data")
        b = self.buf[self.pos]
        self.pos += 1
        return b

    def varint(self):
        shift = result = 0
        while True:
            b = self.byte()
            result |= (b & 0x7F) << shift
            if not b & 0x80:
                return result
            shift += 7
            if shift > 70:
                raise ThriftError("varint too long")

    def zigzag(self):
        n = self.varint()
        return (n >> 1) ^ -(n & 1)

    def skip(self, t):
        if t in (T_TRUE, T_FALSE):
            return
        if t == T_BYTE:
            self.byte()
        elif t in (T_I16, T_I32, T_I64):
            self.varint()
        elif t == T_DOUBLE:
            self.pos += 8
        elif t == T_BINARY:
            n = self.varint()
            self.pos += n
        elif t in (T_LIST, T_SET):
            h = self.byte()
            n = h >> 4
            if n == 15:
                n = self.varint()
            et = h & 0x0F
            for _ in range(n):
                self.skip(et)
        elif t == T_MAP:
            n = self.varint()
            if n:
                kv = self.byte()
                for _ in range(n):
                    self.skip(kv >> 4)
                    self.skip(kv & 0x0F)
        elif t == T_STRUCT:
            self.struct(lambda fid, ft, r: False)
        else:
            raise ThriftError(f"unknown thrift type {t}")

    def struct(self, on_field):
        """Iterate fields; on_field(fid, type, reader) returns True if it consumed the value."""
        last = 0
        while True:
            h = self.byte()
            t = h & 0x0F
            if t == T_STOP:
                return
            delta = h >> 4
            fid = last + delta if delta else self.zigzag()
            last = fid
            if not on_field(fid, t, self):
                self.skip(t)


def _bool(t):
    return t == T_TRUE


def read_page_header(buf, pos):
    """Parse one PageHeader at `pos`; returns (header dict, position after it)."""
    r = _Reader(buf, pos)
    h = {}

    def sub(fields):
        def on(fid, t, rr):
            name = fields.get(fid)
            if name is None:
                return False
            if t in (T_TRUE, T_FALSE):
                h[name] = _bool(t)
            elif t in (T_I32, T_I16, T_I64):
                h[name] = rr.zigzag()
            else:
                return False
            return True
        return on

    def top(fid, t, rr):
        if fid == 1 and t == T_I32:
            h["type"] = rr.zigzag()
        elif fid == 2 and t == T_I32:
            h["uncompressed_page_size"] = rr.zigzag()
        elif fid == 3 and t == T_I32:
            h["compressed_page_size"] = rr.zigzag()
        elif fid == 4 and t == T_I32:
            h["crc"] = rr.zigzag()
        elif fid == 5 and t == T_STRUCT:   # DataPageHeader
            rr.struct(sub({1: "num_values", 2: "encoding", 3: "definition_level_encoding",
                           4: "repetition_level_encoding"}))
        elif fid == 7 and t == T_STRUCT:   # DictionaryPageHeader
            rr.struct(sub({1: "num_values", 2: "encoding", 3: "is_sorted"}))
        elif fid == 8 and t == T_STRUCT:   # DataPageHeaderV2
            rr.struct(sub({1: "num_values", 2: "num_nulls", 3: "num_rows", 4: "encoding",
                           5: "definition_levels_byte_length", 6: "repetition_levels_byte_length",
                           7: "is_compressed"}))
        else:
            return False
        return True

    r.struct(top)
    for k in ("type", "compressed_page_size"):
        if k not in h:
            raise ThriftError(f"PageHeader missing required field {k}")
    return h, r.pos


def read_column_chunk(buf, start, length, physical_type, max_def=0, max_rep=0, type_length=0, num_values=None,
                      codec=0):
    """Split an uncompressed column chunk [start, start+length) into a ColumnChunk.

    Mirrors ParquetFileReader.Chunk.readAllPages (:1824-1979): DICTIONARY_PAGE ->
    the chunk's dictionary, DATA_PAGE -> DataPageV1, DATA_PAGE_V2 -> DataPageV2
    (level sections located by their byte lengths), INDEX_PAGE skipped.
    """
    chunk = ColumnChunk(physical_type=physical_type, max_rep=max_rep, max_def=max_def, type_length=type_length)
    pos, end = start, start + length
    seen = 0
    while pos < end and (num_values is None or seen < num_values):
        h, body = read_page_header(buf, pos)
        size = h["compressed_page_size"]
        usize = h.get("uncompressed_page_size", size)
        if codec not in (0, 1, 2, 6, 7):
            raise ThriftError(f"codec {codec} is not supported (UNCOMPRESSED, SNAPPY, GZIP, ZSTD and LZ4_RAW are)")
        # UNCOMPRESSED: CodecFactory.NO_OP_DECOMPRESSOR hands the page bytes on as they are, whatever
        # uncompressed_page_size says (CodecFactory.java:60-83); the codec alone decides (pqg_pages_from_headers)
        data = bytes(buf[body:body + size])
        if len(data) != size:
            raise ThriftError("page body truncated")
        t = h["type"]
        if t == DICTIONARY_PAGE:
            chunk.dict_page = data
            chunk.dict_num_values = h["num_values"]
            chunk.dict_encoding = h["encoding"]
            if codec:
                chunk.dict_codec, chunk.dict_uncompressed_size = codec, usize
        elif t == DATA_PAGE:
            chunk.pages.append(Page(body=data, num_values=h["num_values"], encoding=h["encoding"], version=1,
                                    rl_encoding=h["repetition_level_encoding"],
                                    dl_encoding=h["definition_level_encoding"], codec=codec,
                                    uncompressed_size=usize if codec else 0))
            seen += h["num_values"]
        elif t == DATA_PAGE_V2:
            compressed = bool(codec) and h.get("is_compressed", True)
            chunk.pages.append(Page(body=data, num_values=h["num_values"], encoding=h["encoding"], version=2,
                                    rl_byte_length=h["repetition_levels_byte_length"],
                                    dl_byte_length=h["definition_levels_byte_length"],
                                    num_nulls=h.get("num_nulls", 0), num_rows=h.get("num_rows", 0),
                                    codec=codec if compressed else 0, uncompressed_size=usize if compressed else 0))
            seen += h["num_values"]
        pos = body + size
    return chunk


def read_footer_length(buf):
    if bytes(buf[-4:]) != b"PAR1":
        raise ThriftError("not a parquet file")
    return struct.unpack("<i", bytes(buf[-8:-4]))[0]


TYPE_BY_NAME = {v: k for k, v in abi.TYPE_NAMES.items()}


def frame_chunk_native(chunk_bytes, value_count=-1, verify_crc=True):
    """The C-ABI page framing (pqg_frame_chunk, host code of libpqgpu.so) over raw chunk bytes.
    Returns (rc, status, [abi.PageHeader, ...])."""
    import ctypes as C

    import numpy as np

    from . import native
    buf = np.frombuffer(bytes(chunk_bytes), dtype=np.uint8)
    L = native.lib()
    n = C.c_int(0)
    st = abi.Status()
    cap = 64
    while True:
        hdrs = (abi.PageHeader * cap)()
        rc = L.pqg_frame_chunk(buf.ctypes.data if buf.size else None, buf.size, value_count, int(bool(verify_crc)),
                               C.addressof(hdrs), cap, C.byref(n), C.byref(st))
        if rc == abi.ERR_INVALID_ARG and n.value > cap:
            cap = n.value
            continue
        return rc, st, [hdrs[i] for i in range(min(n.value, cap))]
