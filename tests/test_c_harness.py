"""The boundary driven from C (tests/c/harness.c, compiled with gcc against include/ and
libpqgpu.so — no ctypes): raw chunk bytes -> pqg_frame_chunk -> pqg_pages_from_headers ->
pqg_decode_host -> per-page pqg_values_reader (initFromPage, readX, skip(n), readValueDictionaryId),
every failure mapped to the Java exception class the JNI shim throws. Mirrors the ValuesReader
contract pinned by TestValuesReaderImpl (parquet-column/src/test/java/org/apache/parquet/column/values/
TestValuesReaderImpl.java) and the readers' error behaviour."""
import os
import struct
import subprocess
import zlib

import numpy as np
import pytest

import fixtures
import thrift_compact
from pqgpu import abi, native, writer

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS_SRC = os.path.join(REPO, "tests", "c", "harness.c")


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("harness") / "harness")
    libdir = os.path.dirname(native.LIB_PATH)
    subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(REPO, "include"),
                    HARNESS_SRC, "-o", exe, "-L", libdir, "-l:libpqgpu.so", f"-Wl,-rpath,{libdir}"], check=True)
    return exe


def case_file(tmp_path, raw, ptype, num_values, type_length=0, max_def=0, max_rep=0, flags=0, codec=0):
    p = tmp_path / "case.bin"
    p.write_bytes(b"PQGC" + struct.pack("<6i", ptype, type_length, max_def, max_rep, flags, codec) +
                  struct.pack("<qQ", num_values, len(raw)) + raw)
    return str(p)


def run(harness, case, mode="all"):
    out = subprocess.run([harness, case, mode], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return out.stdout.splitlines()


def parse(lines):
    """-> dict: frame / decode / per-page values / page ends / init errors."""
    res = {"values": {}, "ends": {}, "init": {}, "pages": {}}
    for ln in lines:
        f = ln.split()
        if f[0] == "V":
            res["values"].setdefault(int(f[1]), []).append((int(f[2]), f[3]))
        elif f[0] == "END":
            res["ends"][int(f[1])] = (int(f[2]), f[3])
        elif f[0] == "PAGE" and f[2] == "INIT_ERROR":
            res["init"][int(f[1])] = (int(f[3]), f[4])
        elif f[0] == "PAGE":
            res["pages"][int(f[1])] = int(f[2])
        else:
            res[f[0]] = f[1:]
    return res


def fmt(v, ptype):
    if ptype in (abi.INT32, abi.INT64, abi.BOOLEAN):
        return str(int(v))
    if ptype == abi.FLOAT:
        return "%08x" % np.float32(v).view(np.uint32)
    if ptype == abi.DOUBLE:
        return "%016x" % np.float64(v).view(np.uint64)
    b = bytes(v)
    return b.hex() if b else "-"


def raw_chunk(name, c):
    buf = np.fromfile(os.path.join(fixtures.GOLDEN, name + ".parquet"), dtype=np.uint8).tobytes()
    return buf[c["start"]: c["start"] + c["length"]]


def required_cases():
    out = []
    for name, c in fixtures.chunk_cases():
        if c["max_def"] == 0 and c["max_rep"] == 0 and c.get("compression", "UNCOMPRESSED") == "UNCOMPRESSED" \
                and c["num_values"] > 0:
            out.append((name, c))
    return out


# ---- CPU: builds, frames, maps errors without a device -----------------------------------

@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="checks the no-device behaviour")
def test_harness_without_device(harness, tmp_path):
    name, c = required_cases()[0]
    ch, _ = fixtures.load_chunk(name, c)
    r = parse(run(harness, case_file(tmp_path, raw_chunk(name, c), ch.physical_type, c["num_values"])))
    assert int(r["FRAME"][0]) >= 1
    assert r["CTX_ERROR"] == [str(abi.ERR_NO_DEVICE), "java/lang/IllegalStateException"]


def test_harness_crc_failure_is_a_parquet_decoding_exception(harness, tmp_path):
    for name, c in fixtures.chunk_cases():
        if name.startswith("test-append"):
            raw = bytearray(raw_chunk(name, c))
            raw[-3] ^= 0x10  # inside the last page's body
            ch, _ = fixtures.load_chunk(name, c)
            r = parse(run(harness, case_file(tmp_path, bytes(raw), ch.physical_type, c["num_values"])))
            assert r["FRAME_ERROR"][:2] == [str(abi.ERR_CRC), "org/apache/parquet/io/ParquetDecodingException"]
            return
    pytest.fail("no CRC fixture")


def test_exception_mapping():
    import ctypes as C
    L = native.lib()
    L.pqg_java_exception.restype = C.c_char_p
    L.pqg_java_exception.argtypes = [C.c_int]
    assert L.pqg_java_exception(abi.OK) is None
    want = {abi.ERR_UNSUPPORTED: "java/lang/UnsupportedOperationException",
            abi.ERR_DICT_ID: "java/lang/ArrayIndexOutOfBoundsException",
            abi.ERR_RLE_PAST_END: "java/lang/IllegalArgumentException",
            abi.ERR_BIT_WIDTH: "java/lang/IllegalArgumentException",
            abi.ERR_EOF: "org/apache/parquet/io/ParquetDecodingException",
            abi.ERR_DELTA_PAST_END: "org/apache/parquet/io/ParquetDecodingException",
            abi.ERR_CRC: "org/apache/parquet/io/ParquetDecodingException",
            abi.ERR_NO_DEVICE: "java/lang/IllegalStateException"}
    for code, cls in want.items():
        assert L.pqg_java_exception(code).decode() == cls


# ---- GPU: values through the C reader -----------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["all", "skip"])
@pytest.mark.parametrize("name,c", required_cases(), ids=lambda x: x if isinstance(x, str) else x["key"])
def test_harness_reads_fixture_values(harness, tmp_path, name, c, mode):
    ch, expected = fixtures.load_chunk(name, c)
    r = parse(run(harness, case_file(tmp_path, raw_chunk(name, c), ch.physical_type, c["num_values"],
                                     type_length=ch.type_length), mode))
    assert r["DECODE"][0] == "0"
    assert r["REFUSED_WRONG_TYPE"] == ["1"]
    pos = 0
    for p in sorted(r["pages"]):
        n = r["pages"][p]
        got = r["values"].get(p, [])
        want_idx = list(range(n)) if mode == "all" else [k for k in range(n) if k % 5 >= 3]
        assert [k for k, _ in got] == want_idx
        for k, v in got:
            assert v == fmt(expected[pos + k], ch.physical_type), (p, k)
        # the read after the page's last value: EOF -> ParquetDecodingException
        assert r["ends"][p] == (abi.ERR_EOF, "org/apache/parquet/io/ParquetDecodingException")
        pos += n
    assert pos == len(expected)


def dict_plain(ch):
    """PLAIN dictionary page -> values (test-side decode of a fixed-width dictionary)."""
    w = abi.elem_width(ch.physical_type, ch.type_length)
    return np.frombuffer(ch.dict_page[: ch.dict_num_values * w], dtype=abi.numpy_dtype(ch.physical_type))


@pytest.mark.gpu
def test_harness_dictionary_ids(harness, tmp_path):
    """PQG_COLUMN_DICTIONARY_IDS: readValueDictionaryId gives the ids; dictionary[ids] == the values."""
    done = 0
    for name, c in fixtures.chunk_cases():
        ch, expected = fixtures.load_chunk(name, c)
        if fixtures.is_compressed(ch) or c["num_values"] == 0 or ch.dict_page is None or \
                ch.physical_type not in (abi.INT32, abi.INT64, abi.DOUBLE, abi.FLOAT):
            continue
        if any(pg.encoding not in (abi.RLE_DICTIONARY, abi.PLAIN_DICTIONARY) for pg in ch.pages):
            continue
        r = parse(run(harness, case_file(tmp_path, raw_chunk(name, c), ch.physical_type, c["num_values"],
                                         max_def=c["max_def"], max_rep=c["max_rep"], flags=abi.COLUMN_DICTIONARY_IDS)))
        assert r["DECODE"][0] == "0" and r["REFUSED_WRONG_TYPE"] == ["1"]
        ids = np.array([int(v) for p in sorted(r["values"]) for _, v in r["values"][p]])
        d = dict_plain(ch)
        assert np.array_equal(d[ids].view(np.uint8), np.asarray(expected).view(np.uint8))
        done += 1
    # synthetic: ids are exactly what the writer assigned (first-appearance order)
    rng = np.random.default_rng(3)
    vals = rng.integers(0, 300, size=50000).astype(np.int64) * 7
    ch = writer.write_column_chunk(abi.INT64, vals, abi.RLE_DICTIONARY, page_rows=7000)
    ids_w, dv = writer.dictionary_encode(vals)
    raw = thrift_compact.chunk_bytes(ch)
    r = parse(run(harness, case_file(tmp_path, raw, abi.INT64, len(vals), flags=abi.COLUMN_DICTIONARY_IDS)))
    ids = [int(v) for p in sorted(r["values"]) for _, v in r["values"][p]]
    assert ids == ids_w.tolist()
    assert done >= 10


@pytest.mark.gpu
def test_harness_ids_on_plain_page_unsupported(harness, tmp_path):
    ch = writer.write_column_chunk(abi.INT64, np.arange(100, dtype=np.int64), abi.PLAIN)
    r = parse(run(harness, case_file(tmp_path, thrift_compact.chunk_bytes(ch), abi.INT64, 100,
                                     flags=abi.COLUMN_DICTIONARY_IDS)))
    assert r["DECODE"][:2] == [str(abi.ERR_UNSUPPORTED), "java/lang/UnsupportedOperationException"]
    assert r["init"][0] == (abi.ERR_UNSUPPORTED, "java/lang/UnsupportedOperationException")


@pytest.mark.gpu
def test_harness_value_error_surfaces_at_the_failing_read(harness, tmp_path):
    """A dictionary id past the dictionary (header claims fewer entries): the reads before it
    succeed, the failing read throws ArrayIndexOutOfBoundsException (Dictionary.decodeToLong), later
    pages are not served."""
    rng = np.random.default_rng(9)
    vals = rng.integers(0, 40, size=30000).astype(np.int64)
    ch = writer.write_column_chunk(abi.INT64, vals, abi.RLE_DICTIONARY, page_rows=10000)
    ids, _ = writer.dictionary_encode(vals)
    limit = 35
    bad = int(np.argmax(ids >= limit))
    raw = thrift_compact.chunk_bytes(ch, dict_num_values=limit)
    r = parse(run(harness, case_file(tmp_path, raw, abi.INT64, len(vals))))
    page, idx = bad // 10000, bad % 10000
    assert r["DECODE"] == [str(abi.ERR_DICT_ID), "java/lang/ArrayIndexOutOfBoundsException", str(page), str(idx)]
    got = r["values"].get(page, [])
    assert len(got) == idx and all(v == str(int(vals[page * 10000 + k])) for k, v in got)
    assert r["ends"][page] == (abi.ERR_DICT_ID, "java/lang/ArrayIndexOutOfBoundsException")
    for p in range(page + 1, 3):
        assert r["init"][p][0] == abi.ERR_DICT_ID


# ---- the chunk codec decides compression (ColumnChunkPageReadStore.readPage) ---------------------

def _chunk(version, n=3000, dict_enc=False):
    vals = np.arange(n, dtype=np.int64) * 3 - 7
    if dict_enc:
        return vals % 50, writer.write_column_chunk(abi.INT64, vals % 50, abi.RLE_DICTIONARY, page_rows=1000,
                                                    version=version)
    return vals, writer.write_column_chunk(abi.INT64, vals, abi.PLAIN, page_rows=1000, version=version)


@pytest.mark.parametrize("codec", [abi.CODEC_SNAPPY, abi.CODEC_ZSTD, abi.CODEC_GZIP])
def test_codec_v1_page_with_equal_sizes_is_compressed(harness, tmp_path, codec):
    """A V1 page of a compressed chunk goes through the decompressor whatever its header sizes say
    (ColumnChunkPageReadStore.java:147-181): equal compressed / uncompressed sizes must not make
    pqg_pages_from_headers describe its bytes as values. -> UNSUPPORTED (decompress first)."""
    vals, ch = _chunk(1)
    raw = thrift_compact.chunk_bytes(ch)
    r = parse(run(harness, case_file(tmp_path, raw, abi.INT64, len(vals), codec=codec)))
    assert r["FRAME_ERROR"][:3] == [str(abi.ERR_UNSUPPORTED), "java/lang/UnsupportedOperationException", "0"]


def test_codec_dictionary_page_of_compressed_chunk(harness, tmp_path):
    """The dictionary page is decompressed with the chunk codec (readDictionaryPage :313-316)."""
    vals, ch = _chunk(2, dict_enc=True)
    raw = thrift_compact.chunk_bytes(ch)
    r = parse(run(harness, case_file(tmp_path, raw, abi.INT64, len(vals), codec=abi.CODEC_SNAPPY)))
    assert r["FRAME_ERROR"][:3] == [str(abi.ERR_UNSUPPORTED), "java/lang/UnsupportedOperationException", "0"]


def test_codec_v2_is_compressed_flag_decides(harness, tmp_path):
    """V2: is_compressed=true with equal sizes in a SNAPPY chunk -> compressed (UNSUPPORTED here);
    is_compressed=false in a SNAPPY chunk -> the page is taken as it is (:218)."""
    vals, ch = _chunk(2)
    raw = thrift_compact.chunk_bytes(ch, is_compressed=True)
    r = parse(run(harness, case_file(tmp_path, raw, abi.INT64, len(vals), codec=abi.CODEC_SNAPPY)))
    assert r["FRAME_ERROR"][:3] == [str(abi.ERR_UNSUPPORTED), "java/lang/UnsupportedOperationException", "0"]
    raw = thrift_compact.chunk_bytes(ch, is_compressed=False)
    r = parse(run(harness, case_file(tmp_path, raw, abi.INT64, len(vals), codec=abi.CODEC_SNAPPY)))
    assert "FRAME_ERROR" not in r and int(r["FRAME"][0]) == len(ch.pages)


def test_codec_out_of_range_is_invalid(harness, tmp_path):
    vals, ch = _chunk(1)
    r = parse(run(harness, case_file(tmp_path, thrift_compact.chunk_bytes(ch), abi.INT64, len(vals), codec=8)))
    assert r["FRAME_ERROR"][0] == str(abi.ERR_INVALID_ARG)


@pytest.mark.gpu
@pytest.mark.parametrize("version", [1, 2])
def test_codec_uncompressed_pages_decode(harness, tmp_path, version):
    """UNCOMPRESSED chunk (V1 / V2) and a V2 page with is_compressed=false inside a SNAPPY chunk:
    framed and decoded through the C ABI, values equal the written ones."""
    vals, ch = _chunk(version)
    for codec in ([abi.CODEC_UNCOMPRESSED] if version == 1 else [abi.CODEC_UNCOMPRESSED, abi.CODEC_SNAPPY]):
        raw = thrift_compact.chunk_bytes(ch, is_compressed=False)
        r = parse(run(harness, case_file(tmp_path, raw, abi.INT64, len(vals), codec=codec)))
        assert r["DECODE"][0] == "0"
        got = [int(v) for p in sorted(r["values"]) for _, v in r["values"][p]]
        assert got == vals.tolist()
