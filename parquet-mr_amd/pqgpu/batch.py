"""Page-batch layout: the column-chunk / page descriptions and the one-buffer layout that the
decoder uploads (pqg_page_desc / pqg_column_desc tables, 16-byte aligned page bodies).

These are the host-side inputs of `pqgpu.decoder` (and of `pqgpu.framing`, which builds
ColumnChunks from raw Thrift-framed chunk bytes). Synthesizing pages (the restated parquet-mr
encoders) lives outside the product package, in tools/synth/writer.py.
"""
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

from . import abi


@dataclass
class Page:
    body: bytes
    num_values: int
    encoding: int
    version: int = 1
    rl_encoding: int = abi.RLE
    dl_encoding: int = abi.RLE
    rl_byte_length: int = 0
    dl_byte_length: int = 0
    num_nulls: int = 0
    num_rows: int = 0
    # page codec (parquet CompressionCodec: 0 UNCOMPRESSED, 1 SNAPPY). A compressed V1 body is
    # one Snappy block of the whole page; a compressed V2 body is the level sections as they
    # are, then one Snappy block of the data section. uncompressed_size: the header's
    # uncompressed_page_size (V2: levels included).
    codec: int = 0
    uncompressed_size: int = 0


@dataclass
class ColumnChunk:
    physical_type: int
    max_rep: int = 0
    max_def: int = 0
    type_length: int = 0
    pages: List[Page] = field(default_factory=list)
    dict_page: Optional[bytes] = None
    dict_num_values: int = 0
    dict_encoding: int = abi.PLAIN
    dict_codec: int = 0               # codec of the dictionary page (its uncompressed size below)
    dict_uncompressed_size: int = 0
    # expected decode (what the reference reader returns), for tests
    values: Optional[object] = None
    def_levels: Optional[np.ndarray] = None
    rep_levels: Optional[np.ndarray] = None
    # CorruptDeltaByteArrays.requiresSequentialReads(created_by, DELTA_BYTE_ARRAY): build_batch flags
    # the chunk's DELTA_BYTE_ARRAY pages after its first page PQG_PAGE_DBA_CARRY
    dba_carry: bool = False

    @property
    def num_slots(self):
        return sum(p.num_values for p in self.pages)


@dataclass
class PageBatch:
    """All pages of several column chunks in one byte buffer + descriptor tables."""
    data: np.ndarray            # uint8, padded
    pages: np.ndarray           # PAGE_DTYPE
    columns: List[dict]         # pqg_column_desc fields without output pointers
    chunks: List[ColumnChunk]
    page_slot_offsets: np.ndarray  # per page: first slot within its column
    column_slots: List[int]
    column_values: List[int]

    @property
    def n_pages(self):
        return len(self.pages)


ALIGN = 16
PAD = 256


def build_batch(chunks, align=ALIGN):
    """Lay chunks out in one buffer (each page 16-B aligned), build the descriptor tables.

    Several chunks may belong to the same output column (row groups of one column):
    pass `column_of` on the chunk objects via attribute `column_index` to merge.
    """
    pieces = []
    pos = 0

    def place(b):
        nonlocal pos
        off = (pos + align - 1) // align * align
        pieces.append((off, b))
        pos = off + len(b)
        return off

    # output columns: chunks with the same column_index share one output column
    col_index = []
    columns = []
    seen = {}
    for i, ch in enumerate(chunks):
        key = getattr(ch, "column_index", i)
        if key not in seen:
            seen[key] = len(columns)
            columns.append(None)
        col_index.append(seen[key])
    page_rows = []
    slot_off = []
    col_slots = [0] * len(columns)
    col_vals = [0] * len(columns)
    dict_info = {}
    for ci, ch in enumerate(chunks):
        oc = col_index[ci]
        doff = -1
        if ch.dict_page is not None:
            doff = place(ch.dict_page)
        dict_info.setdefault(oc, []).append(doff)
        if columns[oc] is None:
            columns[oc] = dict(physical_type=ch.physical_type, type_length=ch.type_length, max_rep=ch.max_rep,
                               max_def=ch.max_def, dict_offset=doff,
                               dict_size=len(ch.dict_page) if ch.dict_page is not None else 0,
                               dict_num_values=ch.dict_num_values, dict_encoding=ch.dict_encoding)
        elif ch.dict_page is not None:
            raise ValueError("a pqg_column_desc has one dictionary: decode row groups with separate "
                             "dictionaries as separate columns (one per row group)")
        for k, pg in enumerate(ch.pages):
            off = place(pg.body)
            carry = abi.PAGE_DBA_CARRY if (getattr(ch, "dba_carry", False) and k > 0 and
                                           pg.encoding == abi.DELTA_BYTE_ARRAY) else 0
            # V2 pages carry the header's null count (a hint the decoder verifies against the levels)
            nulls_flag = abi.PAGE_NULL_COUNT if pg.version == 2 else 0
            page_rows.append((off, len(pg.body), pg.num_values, oc, pg.version, pg.encoding, pg.rl_encoding,
                              pg.dl_encoding, pg.rl_byte_length, pg.dl_byte_length, carry | nulls_flag,
                              pg.num_nulls if pg.version == 2 else 0, 0))
            slot_off.append(col_slots[oc])
            col_slots[oc] += pg.num_values
        col_vals[oc] += len(ch.values) if ch.values is not None else getattr(ch, "n_values_hint", 0)
    total = pos + PAD
    data = np.zeros((total + align - 1) // align * align, dtype=np.uint8)
    for off, b in pieces:
        data[off:off + len(b)] = np.frombuffer(b, dtype=np.uint8)
    pages = np.array(page_rows, dtype=abi.PAGE_DTYPE) if page_rows else np.zeros(0, dtype=abi.PAGE_DTYPE)
    return PageBatch(data=data, pages=pages, columns=columns, chunks=list(chunks),
                     page_slot_offsets=np.array(slot_off, dtype=np.int64), column_slots=col_slots,
                     column_values=col_vals)


UNCOMPRESSED, SNAPPY, GZIP, ZSTD, LZ4_RAW = 0, 1, 2, 6, 7   # parquet.thrift CompressionCodec
