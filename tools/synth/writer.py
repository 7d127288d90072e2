"""Page writer: synthesizes parquet-mr-identical column chunks (test / bench input).

The encoders are restated in C++ (tools/synth/pqwriter.cpp -> tools/synth/libpqwriter.so) from
parquet-mr's writers; this module assembles their output into data pages the
way parquet-mr's column writers do:

  * V1 pages: [rl section][dl section][data]; RLE level sections carry the
    4-byte little-endian length prefix written by
    RunLengthBitPackingHybridValuesWriter.getBytes (rle/RunLengthBitPackingHybridValuesWriter.java:62-72);
    max level 0 writes nothing (ParquetProperties.java:162-190, ColumnWriterV1.java:60-78).
  * V2 pages: levels without length prefix, byte lengths in the header
    (ColumnWriterV2.java:42-110).
  * Dictionary: ids assigned in first-appearance order (DictionaryValuesWriter.java:
    Plain*DictionaryValuesWriter.write*), data section = 1-byte bit width +
    RLE/bit-packed ids (DictionaryValuesWriter.getBytes :159-186); dictionary
    page = PLAIN values.

The writer is input synthesis only; it is not part of the decode path (the page-batch layout the
decoder uploads is pqgpu.batch, re-exported here for the tests and tools).
"""
import ctypes as C
import os
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from pqgpu import abi
from pqgpu.batch import (ALIGN, GZIP, LZ4_RAW, PAD, SNAPPY, UNCOMPRESSED, ZSTD, ColumnChunk,  # noqa: F401
                          Page, PageBatch, build_batch)

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        # input synthesis only (the restated parquet-mr encoders), built outside the product package
        path = os.path.join(_HERE, "libpqwriter.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run __graft_entry__.build()")
        lib = C.CDLL(path)
        i64, vp = C.c_int64, C.c_void_p
        lib.pqw_rle_encode.argtypes = [C.c_int, vp, i64, vp, i64]
        lib.pqw_rle_encode.restype = i64
        lib.pqw_rle_encode_u8.argtypes = [C.c_int, vp, i64, vp, i64]
        lib.pqw_rle_encode_u8.restype = i64
        lib.pqw_delta_encode_long.argtypes = [vp, i64, C.c_int, C.c_int, vp, i64]
        lib.pqw_delta_encode_long.restype = i64
        lib.pqw_delta_encode_int.argtypes = [vp, i64, C.c_int, C.c_int, vp, i64]
        lib.pqw_delta_encode_int.restype = i64
        _LIB = lib
    return _LIB


def width_from_max_int(bound):
    """BytesUtils.getWidthFromMaxInt (BytesUtils.java:49-51)."""
    return int(bound).bit_length() if bound >= 0 else 32


def _call_with_buffer(fn, *args, cap):
    out = np.empty(max(cap, 16), dtype=np.uint8)
    n = fn(*args, out.ctypes.data, out.size)
    if n < 0:
        out = np.empty(-n, dtype=np.uint8)
        n = fn(*args, out.ctypes.data, out.size)
    return out[:n].tobytes()


def rle_encode(values, bit_width):
    """RunLengthBitPackingHybridEncoder: <encoded-data> of `values` (no length prefix)."""
    v = np.ascontiguousarray(values, dtype=np.int32)
    cap = 64 + (len(v) // 8 + 2) * (max(bit_width, 9) + 2)
    return _call_with_buffer(_lib().pqw_rle_encode, bit_width, v.ctypes.data, len(v), cap=cap)


def rle_encode_levels(levels, bit_width):
    v = np.ascontiguousarray(levels, dtype=np.uint8)
    cap = 64 + (len(v) // 8 + 2) * (max(bit_width, 9) + 2)
    return _call_with_buffer(_lib().pqw_rle_encode_u8, bit_width, v.ctypes.data, len(v), cap=cap)


def delta_encode(values, physical_type, block=128, miniblocks=4):
    """DeltaBinaryPackingValuesWriterFor{Long,Integer}.getBytes."""
    if physical_type == abi.INT64:
        v = np.ascontiguousarray(values, dtype=np.int64)
        fn = _lib().pqw_delta_encode_long
    else:
        v = np.ascontiguousarray(values, dtype=np.int32)
        fn = _lib().pqw_delta_encode_int
    cap = 64 + len(v) * 9 + (len(v) // block + 1) * (miniblocks + 12)
    return _call_with_buffer(fn, v.ctypes.data, len(v), block, miniblocks, cap=cap)


class BinaryValues:
    """BYTE_ARRAY values as numpy arrays (offsets[n + 1], data) for large synthetic inputs; slices
    like a list of bytes."""

    def __init__(self, offsets, data):
        self.offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        self.data = np.ascontiguousarray(data, dtype=np.uint8)

    @classmethod
    def random(cls, n, min_len, max_len, seed, alphabet=b"abcdefghijklmnopqrstuvwxyz0123456789"):
        rng = np.random.default_rng(seed)
        lens = rng.integers(min_len, max_len + 1, size=n)
        offs = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(lens, out=offs[1:])
        a = np.frombuffer(alphabet, dtype=np.uint8)
        return cls(offs, a[rng.integers(0, a.size, size=int(offs[-1]), dtype=np.uint8)])

    def __len__(self):
        return self.offsets.size - 1

    def lengths(self):
        return np.diff(self.offsets)

    def __getitem__(self, k):
        if isinstance(k, slice):
            a, b, _ = k.indices(len(self))
            o = self.offsets[a:b + 1]
            return BinaryValues(o - o[0], self.data[o[0]:o[-1]])
        return self.data[self.offsets[k]:self.offsets[k + 1]].tobytes()

    def __iter__(self):
        for i in range(len(self)):
            yield self[i]


def _plain_binary_np(v):
    """[4-byte LE length][bytes] per value, vectorized (BinaryValues)."""
    n = len(v)
    lens = v.lengths()
    out = np.empty(4 * n + v.data.size, dtype=np.uint8)
    starts = v.offsets[:-1] + 4 * np.arange(n, dtype=np.int64)  # where each length prefix goes
    lb = lens.astype("<u4").view(np.uint8).reshape(n, 4)
    for k in range(4):
        out[starts + k] = lb[:, k]
    owner = np.repeat(np.arange(n, dtype=np.int64), lens)
    out[np.arange(v.data.size, dtype=np.int64) + 4 * (owner + 1)] = v.data
    return out.tobytes()


def plain_encode(values, physical_type, type_length=0):
    """PlainValuesWriter / BooleanPlainValuesWriter / FixedLenByteArrayPlainValuesWriter."""
    if physical_type == abi.BOOLEAN:
        bits = np.ascontiguousarray(values, dtype=np.uint8) & 1
        return np.packbits(bits, bitorder="little").tobytes()
    if physical_type == abi.BYTE_ARRAY and isinstance(values, BinaryValues):
        return _plain_binary_np(values)
    if physical_type == abi.BYTE_ARRAY:
        out = bytearray()
        for b in values:
            out += len(b).to_bytes(4, "little") + bytes(b)
        return bytes(out)
    if physical_type in (abi.INT96, abi.FIXED_LEN_BYTE_ARRAY):
        w = abi.elem_width(physical_type, type_length)
        return b"".join(bytes(b)[:w].ljust(w, b"\0") for b in values)
    return np.ascontiguousarray(values, dtype=abi.numpy_dtype(physical_type)).tobytes()


def dlba_encode(values):
    """DeltaLengthByteArrayValuesWriter.getBytes (deltalengthbytearray/DeltaLengthByteArrayValuesWriter.java:77-86):
    DELTA_BINARY_PACKED int lengths (128 / 4), then the concatenated bytes."""
    if isinstance(values, BinaryValues):
        return delta_encode(values.lengths().astype(np.int32), abi.INT32) + values.data.tobytes()
    vals = [bytes(b) for b in values]
    lens = np.array([len(b) for b in vals], dtype=np.int32)
    return delta_encode(lens, abi.INT32) + b"".join(vals)


def dba_encode(values, previous=b""):
    """DeltaByteArrayWriter.writeBytes / getBytes (deltastrings/DeltaByteArrayWriter.java:56-58, 90-100):
    prefix lengths shared with the previous value (DELTA_BINARY_PACKED), then the suffixes as
    DELTA_LENGTH_BYTE_ARRAY. `previous` starts empty on every page (reset :65-70); a non-empty
    `previous` writes the page as parquet-mr < 1.8 did (PARQUET-246: reset kept the last value)."""
    if isinstance(values, BinaryValues) and len(values) > 1 and not previous:
        # vectorized: values padded into rows, prefix = first mismatch with the previous row
        lens = values.lengths()
        L = int(lens.max()) + 1
        n = len(values)
        rows = np.zeros((n, L), dtype=np.int16) - 1
        owner = np.repeat(np.arange(n), lens)
        col = np.arange(values.data.size) - np.repeat(values.offsets[:-1], lens)
        rows[owner, col] = values.data
        neq = rows[1:] != rows[:-1]
        pre = np.zeros(n, dtype=np.int32)
        pre[1:] = np.where(neq.any(axis=1), np.argmax(neq, axis=1), L)
        pre[1:] = np.minimum(pre[1:], np.minimum(lens[1:], lens[:-1]))
        keep = np.arange(values.data.size) - np.repeat(values.offsets[:-1], lens) >= np.repeat(pre, lens)
        sfx_lens = (lens - pre).astype(np.int64)
        sfx = BinaryValues(np.concatenate([[0], np.cumsum(sfx_lens)]), values.data[keep])
        return delta_encode(pre, abi.INT32) + dlba_encode(sfx)
    prev = bytes(previous)
    prefixes, suffixes = [], []
    for b in values:
        b = bytes(b)
        n = min(len(prev), len(b))
        i = 0
        while i < n and prev[i] == b[i]:
            i += 1
        prefixes.append(i)
        suffixes.append(b[i:])
        prev = b
    return delta_encode(np.array(prefixes, dtype=np.int32), abi.INT32) + dlba_encode(suffixes)


def bss_encode(values, physical_type, type_length=0):
    """ByteStreamSplitValuesWriter: byte k of value i goes to stream k at index i."""
    w = abi.elem_width(physical_type, type_length)
    if physical_type in (abi.FIXED_LEN_BYTE_ARRAY, abi.INT96):
        raw = np.frombuffer(b"".join(bytes(b)[:w].ljust(w, b"\0") for b in values), dtype=np.uint8)
    else:
        raw = np.ascontiguousarray(values, dtype=abi.numpy_dtype(physical_type)).view(np.uint8)
    return np.ascontiguousarray(raw.reshape(-1, w).T).tobytes()


def dictionary_encode(values):
    """Ids in first-appearance order, as DictionaryValuesWriter assigns them."""
    values = np.asarray(values)
    uniq, first, inverse = np.unique(values, return_index=True, return_inverse=True)
    order = np.argsort(first, kind="stable")
    rank = np.empty_like(order)
    rank[order] = np.arange(len(order))
    ids = rank[inverse.reshape(-1)].astype(np.int32)
    return ids, uniq[order]


def be_pack(values, bit_width):
    """Deprecated BIT_PACKED level encoding (BitPacking / Packer.BIG_ENDIAN): MSB-first bit
    stream, ceil(n * w / 8) bytes."""
    v = np.asarray(values, dtype=np.uint32)
    if bit_width == 0 or v.size == 0:
        return b""
    bits = ((v[:, None] >> np.arange(bit_width - 1, -1, -1, dtype=np.uint32)) & 1).astype(np.uint8).ravel()
    return np.packbits(bits).tobytes()


def _level_section(levels, max_level, version, encoding=abi.RLE):
    if max_level == 0:
        return b""
    if encoding == abi.BIT_PACKED:
        assert version == 1, "BIT_PACKED levels exist only in V1 pages"
        return be_pack(levels, width_from_max_int(max_level))
    body = rle_encode_levels(levels, width_from_max_int(max_level))
    if version == 1:
        return len(body).to_bytes(4, "little") + body
    return body


def _page_bounds(n_slots, page_rows, rep_levels):
    """Slot ranges of each page: `page_rows` slots, closed at record boundaries."""
    bounds = []
    start = 0
    while start < n_slots:
        end = min(start + page_rows, n_slots)
        if rep_levels is not None and end < n_slots:
            while end < n_slots and rep_levels[end] != 0:
                end += 1
        bounds.append((start, end))
        start = end
    if not bounds:
        bounds.append((0, 0))
    return bounds


def write_column_chunk(physical_type, values, encoding, *, def_levels=None, rep_levels=None, max_def=0,
                       max_rep=0, page_rows=20000, version=1, type_length=0, delta_block=128,
                       delta_miniblocks=4, dict_page_encoding=abi.PLAIN, level_encoding=abi.RLE,
                       dba_carry=False):
    """Encode one column chunk. `values` are the non-null values (dense, in slot order).
    dba_carry: DELTA_BYTE_ARRAY pages written like parquet-mr < 1.8 (PARQUET-246: each page's first
    value may share a prefix with the previous page's last value); the chunk is marked so that
    build_batch flags its pages PQG_PAGE_DBA_CARRY."""
    values = values if physical_type == abi.BYTE_ARRAY or physical_type in (abi.INT96, abi.FIXED_LEN_BYTE_ARRAY) \
        else np.asarray(values)
    n_values = len(values)
    if def_levels is None:
        n_slots = n_values
        dl = np.full(n_slots, max_def, dtype=np.uint8)
    else:
        dl = np.asarray(def_levels, dtype=np.uint8)
        n_slots = len(dl)
    rl = np.zeros(n_slots, dtype=np.uint8) if rep_levels is None else np.asarray(rep_levels, dtype=np.uint8)
    nonnull = (dl == max_def)
    assert int(nonnull.sum()) == n_values, "def levels disagree with the value count"
    chunk = ColumnChunk(physical_type=physical_type, max_rep=max_rep, max_def=max_def, type_length=type_length,
                        values=values, def_levels=dl if max_def else None, rep_levels=rl if max_rep else None,
                        dba_carry=dba_carry)
    ids = None
    if encoding in (abi.RLE_DICTIONARY, abi.PLAIN_DICTIONARY):
        if physical_type == abi.BYTE_ARRAY:
            seen = {}
            ids = np.empty(n_values, dtype=np.int32)
            dict_vals = []
            for i, b in enumerate(values):
                b = bytes(b)
                if b not in seen:
                    seen[b] = len(dict_vals)
                    dict_vals.append(b)
                ids[i] = seen[b]
        else:
            ids, dict_vals = dictionary_encode(values)
        chunk.dict_page = plain_encode(dict_vals, physical_type, type_length)
        chunk.dict_num_values = len(dict_vals)
        chunk.dict_encoding = dict_page_encoding
        bit_width = width_from_max_int(len(dict_vals) - 1)
    value_pos = np.concatenate([[0], np.cumsum(nonnull)]).astype(np.int64)
    for (s, e) in _page_bounds(n_slots, page_rows, rl if max_rep else None):
        v0, v1 = int(value_pos[s]), int(value_pos[e])
        if encoding in (abi.RLE_DICTIONARY, abi.PLAIN_DICTIONARY):
            data = bytes([bit_width]) + rle_encode(ids[v0:v1], bit_width)
        elif encoding == abi.PLAIN:
            data = plain_encode(values[v0:v1], physical_type, type_length)
        elif encoding == abi.DELTA_BINARY_PACKED:
            data = delta_encode(values[v0:v1], physical_type, delta_block, delta_miniblocks)
        elif encoding == abi.DELTA_LENGTH_BYTE_ARRAY:
            data = dlba_encode(values[v0:v1])
        elif encoding == abi.DELTA_BYTE_ARRAY:
            data = dba_encode(values[v0:v1], bytes(values[v0 - 1]) if dba_carry and v0 > 0 else b"")
        elif encoding == abi.BYTE_STREAM_SPLIT:
            data = bss_encode(values[v0:v1], physical_type, type_length)
        elif encoding == abi.RLE and physical_type == abi.BOOLEAN:
            # RunLengthBitPackingHybridValuesWriter(1).getBytes: 4-byte LE length + width-1 stream
            rle = rle_encode(np.asarray(values[v0:v1], dtype=np.int32), 1)
            data = len(rle).to_bytes(4, "little") + rle
        else:
            raise ValueError(f"writer does not support encoding {encoding}")
        rls = _level_section(rl[s:e], max_rep, version, level_encoding)
        dls = _level_section(dl[s:e], max_def, version, level_encoding)
        page = Page(body=rls + dls + data, num_values=e - s, encoding=encoding, version=version,
                    rl_encoding=level_encoding, dl_encoding=level_encoding,
                    num_nulls=int((e - s) - (v1 - v0)),
                    num_rows=int((rl[s:e] == 0).sum()) if max_rep else e - s)
        if version == 2:
            page.rl_byte_length, page.dl_byte_length = len(rls), len(dls)
        chunk.pages.append(page)
    return chunk


def write_dict_column_from_ids(physical_type, dict_values, ids, page_rows=20000, encoding=abi.RLE_DICTIONARY,
                               def_levels=None, max_def=0, version=1):
    """Dictionary column from ids already numbered in first-appearance order (fast path for large
    synthetic inputs; same bytes as write_column_chunk). def_levels / max_def: a flat optional column
    (ids are the non-null values' ids; pages of page_rows slots, V1 or V2 level sections)."""
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    bit_width = width_from_max_int(len(dict_values) - 1)
    chunk = ColumnChunk(physical_type=physical_type, values=None, max_def=max_def if def_levels is not None else 0)
    chunk.dict_page = plain_encode(dict_values, physical_type)
    chunk.dict_num_values = len(dict_values)
    if def_levels is None:
        for s in range(0, max(len(ids), 1), page_rows):
            e = min(s + page_rows, len(ids))
            data = bytes([bit_width]) + rle_encode(ids[s:e], bit_width)
            chunk.pages.append(Page(body=data, num_values=e - s, encoding=encoding, num_rows=e - s))
    else:
        dl = np.ascontiguousarray(def_levels, dtype=np.uint8)
        value_pos = np.concatenate([[0], np.cumsum(dl == max_def)]).astype(np.int64)
        assert int(value_pos[-1]) == len(ids)
        for s in range(0, max(len(dl), 1), page_rows):
            e = min(s + page_rows, len(dl))
            v0, v1 = int(value_pos[s]), int(value_pos[e])
            data = bytes([bit_width]) + rle_encode(ids[v0:v1], bit_width)
            dls = _level_section(dl[s:e], max_def, version)
            page = Page(body=dls + data, num_values=e - s, encoding=encoding, version=version,
                        num_nulls=(e - s) - (v1 - v0), num_rows=e - s)
            if version == 2:
                page.dl_byte_length = len(dls)
            chunk.pages.append(page)
    chunk.n_values_hint = len(ids)
    return chunk


def first_appearance_ids(ids):
    """Renumber ids in order of first appearance (DictionaryValuesWriter id assignment)."""
    ids = np.asarray(ids)
    uniq, first = np.unique(ids, return_index=True)
    order = uniq[np.argsort(first, kind="stable")]
    remap = np.empty(int(ids.max()) + 1 if ids.size else 1, dtype=np.int32)
    remap[order] = np.arange(order.size, dtype=np.int32)
    return remap[ids], order


def snappy_chunk(chunk):
    """A copy of `chunk` with every page (and the dictionary page) Snappy-compressed the way
    parquet-mr writes SNAPPY column chunks (V1: the whole body; V2: the data section after the
    level sections). Compression by pyarrow's libsnappy (test-data synthesis only)."""
    import copy

    import pyarrow as pa
    out = copy.deepcopy(chunk)
    if out.dict_page is not None:
        out.dict_uncompressed_size = len(out.dict_page)
        out.dict_page = pa.compress(out.dict_page, codec="snappy", asbytes=True)
        out.dict_codec = SNAPPY
    for pg in out.pages:
        pg.uncompressed_size = len(pg.body)
        lv = pg.rl_byte_length + pg.dl_byte_length if pg.version == 2 else 0
        pg.body = pg.body[:lv] + pa.compress(pg.body[lv:], codec="snappy", asbytes=True)
        pg.codec = SNAPPY
    return out


def zstd_chunk(chunk, level=3):
    """A copy of `chunk` with every page (and the dictionary page) ZSTD-compressed the way
    parquet-mr writes ZSTD column chunks (V1: the whole body; V2: the data section), at parquet-mr's
    default level 3 (ZstandardCodec). Compression by pyarrow's libzstd (test-data synthesis only)."""
    import copy

    import pyarrow as pa
    codec = pa.Codec("zstd", compression_level=level)
    out = copy.deepcopy(chunk)
    if out.dict_page is not None:
        out.dict_uncompressed_size = len(out.dict_page)
        out.dict_page = codec.compress(out.dict_page, asbytes=True)
        out.dict_codec = ZSTD
    for pg in out.pages:
        pg.uncompressed_size = len(pg.body)
        lv = pg.rl_byte_length + pg.dl_byte_length if pg.version == 2 else 0
        pg.body = pg.body[:lv] + codec.compress(pg.body[lv:], asbytes=True)
        pg.codec = ZSTD
    return out


def lz4_raw_chunk(chunk):
    """A copy of `chunk` with every page (and the dictionary page) LZ4_RAW-compressed the way
    parquet-mr writes LZ4_RAW column chunks (Lz4RawCompressor, one raw LZ4 block per page; V1: the
    whole body; V2: the data section after the level sections). Compression by pyarrow's liblz4
    (test-data synthesis only)."""
    import copy

    import pyarrow as pa
    codec = pa.Codec("lz4_raw")
    out = copy.deepcopy(chunk)
    if out.dict_page is not None:
        out.dict_uncompressed_size = len(out.dict_page)
        out.dict_page = codec.compress(out.dict_page, asbytes=True)
        out.dict_codec = LZ4_RAW
    for pg in out.pages:
        pg.uncompressed_size = len(pg.body)
        lv = pg.rl_byte_length + pg.dl_byte_length if pg.version == 2 else 0
        pg.body = pg.body[:lv] + codec.compress(pg.body[lv:], asbytes=True)
        pg.codec = LZ4_RAW
    return out


def gzip_chunk(chunk, level=6):
    """A copy of `chunk` with every page (and the dictionary page) GZIP-compressed the way
    parquet-mr writes GZIP column chunks (Hadoop GzipCodec: one gzip member per page; V1: the whole
    body; V2: the data section). Compression by Python's zlib (test-data synthesis only)."""
    import copy
    import gzip

    out = copy.deepcopy(chunk)
    if out.dict_page is not None:
        out.dict_uncompressed_size = len(out.dict_page)
        out.dict_page = gzip.compress(out.dict_page, compresslevel=level)
        out.dict_codec = GZIP
    for pg in out.pages:
        pg.uncompressed_size = len(pg.body)
        lv = pg.rl_byte_length + pg.dl_byte_length if pg.version == 2 else 0
        pg.body = pg.body[:lv] + gzip.compress(pg.body[lv:], compresslevel=level)
        pg.codec = GZIP
    return out
