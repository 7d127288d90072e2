"""Page framing through the C ABI (pqg_frame_chunk / pqg_pages_from_headers / pqg_crc32, host code of
libpqgpu.so): raw column-chunk bytes of the reference's fixture files in, page headers out, as
ParquetFileReader.Chunk.readAllPages reads them (ParquetFileReader.java:1824-1979), including the
CRC check (verifyCrc :1805-1813). test-append_{1,2}.parquet (written by parquet-mr 1.13) carry
page CRCs; pyarrow-written files with page checksums cover V2 and SNAPPY pages. No GPU needed."""
import ctypes as C
import io
import os
import zlib

import numpy as np
import pytest

import fixtures
from pqgpu import abi, framing, native
from tools.synth import writer
from thrift_compact import page_header


def chunk_bytes(name, c):
    buf = np.fromfile(os.path.join(fixtures.GOLDEN, name + ".parquet"), dtype=np.uint8).tobytes()
    return buf[c["start"]: c["start"] + c["length"]]


@pytest.mark.parametrize("name,c", list(fixtures.chunk_cases()), ids=lambda x: x if isinstance(x, str) else x["key"])
def test_fixture_chunks_match_python_framing(name, c):
    raw = chunk_bytes(name, c)
    rc, st, hdrs = framing.frame_chunk_native(raw, c["num_values"], verify_crc=True)
    assert rc == abi.OK, st.message
    # the Python restatement (used by every fixture decode test) walks the same headers
    pos, exp = 0, []
    seen = 0
    while seen < c["num_values"]:
        h, body = framing.read_page_header(raw, pos)
        if h["type"] in (framing.DICTIONARY_PAGE, framing.DATA_PAGE, framing.DATA_PAGE_V2):
            exp.append((h, pos, body))
            if h["type"] != framing.DICTIONARY_PAGE:
                seen += h["num_values"]
        pos = body + h["compressed_page_size"]
    assert len(hdrs) == len(exp)
    for g, (h, hpos, body) in zip(hdrs, exp):
        assert (g.type, g.compressed_page_size, g.header_offset, g.body_offset) == \
               (h["type"], h["compressed_page_size"], hpos, body)
        assert g.uncompressed_page_size == h.get("uncompressed_page_size", 0)
        assert g.num_values == h["num_values"] and g.encoding == h["encoding"]
        assert bool(g.has_crc) == ("crc" in h)
        if g.type == framing.DATA_PAGE:
            assert g.definition_level_encoding == h["definition_level_encoding"]
            assert g.repetition_level_encoding == h["repetition_level_encoding"]
        if g.type == framing.DATA_PAGE_V2:
            assert g.definition_levels_byte_length == h["definition_levels_byte_length"]
            assert g.repetition_levels_byte_length == h["repetition_levels_byte_length"]
            assert bool(g.is_compressed) == h.get("is_compressed", True)


def crc_fixture_chunks():
    return [(n, c) for n, c in fixtures.chunk_cases() if n.startswith("test-append")]


def test_reference_files_carry_page_crcs():
    n_crc = 0
    for name, c in crc_fixture_chunks():
        rc, st, hdrs = framing.frame_chunk_native(chunk_bytes(name, c), c["num_values"])
        assert rc == abi.OK, st.message
        n_crc += sum(h.has_crc for h in hdrs)
    assert n_crc >= 4  # parquet-mr 1.13 writes page.write.checksum (ParquetProperties default)


@pytest.mark.parametrize("name,c", crc_fixture_chunks(), ids=lambda x: x if isinstance(x, str) else x["key"])
def test_crc_mismatch_names_the_page(name, c):
    raw = bytearray(chunk_bytes(name, c))
    rc, st, hdrs = framing.frame_chunk_native(bytes(raw), c["num_values"])
    for k, h in enumerate(hdrs):
        if not h.has_crc or h.compressed_page_size == 0:
            continue
        bad = bytearray(raw)
        bad[h.body_offset + h.compressed_page_size // 2] ^= 0x40
        rc, st, _ = framing.frame_chunk_native(bytes(bad), c["num_values"])
        assert rc == abi.ERR_CRC and st.page == k, (rc, st.page, k)
        assert b"CRC checksum verification failed" in st.message
        assert (b"dictionary page" in st.message) == (h.type == framing.DICTIONARY_PAGE)
        # verification off (usePageChecksumVerification false): the flipped byte passes framing
        rc, st, _ = framing.frame_chunk_native(bytes(bad), c["num_values"], verify_crc=False)
        assert rc == abi.OK


@pytest.mark.parametrize("version", ["1.0", "2.0"])
@pytest.mark.parametrize("compression", ["NONE", "SNAPPY"])
def test_pyarrow_page_checksums(version, compression):
    pa = pytest.importorskip("pyarrow")
    pq = pytest.importorskip("pyarrow.parquet")
    rng = np.random.default_rng(4)
    t = pa.table({"a": pa.array(rng.integers(0, 50, size=30000)),
                  "s": pa.array([None if i % 7 == 0 else f"v{i % 300}" for i in range(30000)])})
    sink = io.BytesIO()
    pq.write_table(t, sink, data_page_version=version, compression=compression, write_page_checksum=True,
                   data_page_size=16384)
    raw = sink.getvalue()
    md = pq.ParquetFile(io.BytesIO(raw)).metadata
    for ci in range(md.num_columns):
        cm = md.row_group(0).column(ci)
        start = cm.dictionary_page_offset if cm.has_dictionary_page else cm.data_page_offset
        chunk = raw[start: start + cm.total_compressed_size]
        rc, st, hdrs = framing.frame_chunk_native(chunk, cm.num_values)
        assert rc == abi.OK, st.message
        assert all(h.has_crc for h in hdrs) and len(hdrs) >= 2
        for h in hdrs:
            body = chunk[h.body_offset: h.body_offset + h.compressed_page_size]
            assert zlib.crc32(body) == h.crc
        h = hdrs[-1]
        bad = bytearray(chunk)
        bad[h.body_offset] ^= 1
        rc, st, _ = framing.frame_chunk_native(bytes(bad), cm.num_values)
        assert rc == abi.ERR_CRC and st.page == len(hdrs) - 1


def test_crc32_matches_zlib():
    L = native.lib()
    rng = np.random.default_rng(0)
    for n in [0, 1, 7, 8, 9, 63, 64, 1000, 65537]:
        d = rng.integers(0, 256, size=n, dtype=np.uint8)
        assert L.pqg_crc32(0, d.ctypes.data if n else None, n) == zlib.crc32(d.tobytes())
        if n > 10:  # continuation
            c1 = L.pqg_crc32(0, d.ctypes.data, 5)
            assert L.pqg_crc32(c1, d[5:].ctypes.data, n - 5) == zlib.crc32(d.tobytes())



def test_skips_index_pages_and_unknown_fields():
    body = b"\x01" * 10
    raw = (page_header(2, 4, 1, extra_field=True) + b"abcd" + page_header(1, 6, 0) + b"zzzzzz" +
           page_header(0, 10, 5, enc=8) + body + page_header(3, 10, 5, enc=0, v2=(2, 3)) + body)
    rc, st, hdrs = framing.frame_chunk_native(raw, 10)
    assert rc == abi.OK, st.message
    assert [h.type for h in hdrs] == [framing.DICTIONARY_PAGE, framing.DATA_PAGE, framing.DATA_PAGE_V2]
    assert hdrs[2].repetition_levels_byte_length == 2 and hdrs[2].definition_levels_byte_length == 3
    assert hdrs[2].is_compressed == 0


def test_error_paths():
    body = b"\x00" * 8
    good = page_header(0, 8, 4) + body
    # value count reached exactly; more than available -> the next header is missing (EOF)
    assert framing.frame_chunk_native(good, 4)[0] == abi.OK
    rc, st, _ = framing.frame_chunk_native(good, 5)
    assert rc == abi.ERR_EOF
    # fewer values than the pages hold
    rc, st, _ = framing.frame_chunk_native(good + good, 6)
    assert rc == abi.ERR_CORRUPT and b"Expected 6 values" in st.message
    # body past the end
    rc, st, _ = framing.frame_chunk_native(good[:-1], 4)
    assert rc == abi.ERR_EOF
    # truncated header
    rc, st, _ = framing.frame_chunk_native(good[:3], 4)
    assert rc in (abi.ERR_CORRUPT, abi.ERR_EOF)
    # two dictionary pages
    d = page_header(2, 4, 1) + b"abcd"
    rc, st, _ = framing.frame_chunk_native(d + d + good, 4)
    assert rc == abi.ERR_CORRUPT and st.page == 1 and b"more than one dictionary page" in st.message
    # V2 level lengths larger than the page
    rc, st, _ = framing.frame_chunk_native(page_header(3, 8, 4, v2=(5, 5)) + body, 4)
    assert rc == abi.ERR_CORRUPT
    # CRC of a hand-built page
    crc = zlib.crc32(body)
    assert framing.frame_chunk_native(page_header(0, 8, 4, crc=crc) + body, 4)[0] == abi.OK
    rc, st, _ = framing.frame_chunk_native(page_header(0, 8, 4, crc=crc ^ 1) + body, 4)
    assert rc == abi.ERR_CRC


def test_pages_from_headers_match_build_batch():
    """Headers -> pqg_page_desc + the column's dictionary fields == what writer.build_batch lays out
    for the same fixture chunk (so the framed descriptors feed pqg_decode unchanged)."""
    L = native.lib()
    for name, c in fixtures.chunk_cases():
        ch, _ = fixtures.load_chunk(name, c)
        if fixtures.is_compressed(ch):
            continue
        raw = chunk_bytes(name, c)
        rc, st, hdrs = framing.frame_chunk_native(raw, c["num_values"])
        arr = (abi.PageHeader * max(1, len(hdrs)))(*hdrs)
        col = abi.ColumnDesc()
        col.dict_offset = -1
        pages = (abi.PageDesc * max(1, len(hdrs)))()
        n = C.c_int(0)
        base = 4096
        rc = L.pqg_pages_from_headers(C.addressof(arr), len(hdrs), abi.CODEC_UNCOMPRESSED, base, 0, C.byref(col), C.addressof(pages),
                                      len(hdrs), C.byref(n), C.byref(st))
        assert rc == abi.OK, st.message
        assert n.value == len(ch.pages)
        for k, pg in enumerate(ch.pages):
            p = pages[k]
            assert raw[p.offset - base: p.offset - base + p.size] == pg.body
            assert (p.num_values, p.version, p.encoding) == (pg.num_values, pg.version, pg.encoding)
            if pg.version == 2:
                assert (p.rl_byte_length, p.dl_byte_length) == (pg.rl_byte_length, pg.dl_byte_length)
            else:
                assert (p.rl_encoding, p.dl_encoding) == (pg.rl_encoding, pg.dl_encoding)
        if ch.dict_page is not None:
            assert raw[col.dict_offset - base: col.dict_offset - base + col.dict_size] == ch.dict_page
            assert (col.dict_num_values, col.dict_encoding) == (ch.dict_num_values, ch.dict_encoding)
        else:
            assert col.dict_offset == -1
