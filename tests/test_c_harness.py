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
from pqgpu import abi, native
from tools.synth import writer

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS_SRC = os.path.join(REPO, "tests", "c", "harness.c")
ROUTER_SRC = os.path.join(REPO, "tests", "c", "router.c")


def _build(tmp_path_factory, src, name):
    exe = str(tmp_path_factory.mktemp(name) / name)
    libdir = os.path.dirname(native.LIB_PATH)
    subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(REPO, "include"),
                    src, "-o", exe, "-L", libdir, "-l:libpqgpu.so", f"-Wl,-rpath,{libdir}"], check=True)
    return exe


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    return _build(tmp_path_factory, HARNESS_SRC, "harness")


@pytest.fixture(scope="module")
def router(tmp_path_factory):
    return _build(tmp_path_factory, ROUTER_SRC, "router")


def case_file(tmp_path, raw, ptype, num_values, type_length=0, max_def=0, max_rep=0, flags=0, codec=0, name="case.bin"):
    p = tmp_path / name
    p.write_bytes(b"PQGC" + struct.pack("<6i", ptype, type_length, max_def, max_rep, flags, codec) +
                  struct.pack("<qQ", num_values, len(raw)) + raw)
    return str(p)


def run(harness, case, mode="all", more=()):
    out = subprocess.run([harness, case, mode, *more], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    return out.stdout.splitlines()


def parse(lines):
    """-> dict: frame / decode / per-page values / page ends / init errors."""
    res = {"values": {}, "ends": {}, "init": {}, "pages": {}, "levels": {}, "perr": {}, "pagecol": {}}
    for ln in lines:
        f = ln.split()
        if f[0] == "L":
            res["levels"].setdefault(int(f[1]), []).append((int(f[2]), int(f[3]), int(f[4])))
        elif f[0] == "PERR":
            res["perr"][int(f[1])] = (int(f[2]), int(f[3]), int(f[4]))
        elif f[0] == "PAGECOL":
            res["pagecol"][int(f[1])] = int(f[2])
        elif f[0] == "V":
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
@pytest.mark.parametrize("mode", ["all", "skip", "staged"])
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
        want_idx = list(range(n)) if mode in ("all", "staged") else [k for k in range(n) if k % 5 >= 3]
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


# ---- levels through the boundary (pqg_lr_*), per-column error scoping, the staged path ------------

def _c5_chunk(recs=3000, page_rows=1000, version=1, seed=7):
    """C5's shape (LIST<optional int64>: rep + def levels, Poisson(3) lists, 10 % null lists /
    elements), small: the values and the levels the writer wrote."""
    rng = np.random.default_rng(seed)
    lens = rng.poisson(3, size=recs)
    null_list = rng.random(recs) < 0.1
    slots = np.where(null_list | (lens == 0), 1, lens)
    starts = np.concatenate([[0], np.cumsum(slots)[:-1]])
    rl = np.ones(int(slots.sum()), dtype=np.uint8)
    rl[starts] = 0
    dl = np.full(rl.size, 3, dtype=np.uint8)
    dl[rng.random(rl.size) < 0.1] = 2
    dl[starts[null_list]] = 0
    dl[starts[~null_list & (lens == 0)]] = 1
    vals = rng.integers(-2**40, 2**40, size=int((dl == 3).sum()))
    ch = writer.write_column_chunk(abi.INT64, vals, abi.PLAIN, def_levels=dl, rep_levels=rl, max_def=3, max_rep=1,
                                   page_rows=page_rows, version=version)
    return ch, vals, dl, rl


def _level_stream(r, pages):
    """(rep, def) per slot and the values read, in page order, from a levels-mode run."""
    reps, defs, vals = [], [], []
    for p in pages:
        for _, rv, dv in r["levels"].get(p, []):
            reps.append(rv)
            defs.append(dv)
        vals += [v for _, v in r["values"].get(p, [])]
    return np.array(reps, dtype=np.int64), np.array(defs, dtype=np.int64), vals


def _oracle(ch):
    from oracle import pqref
    return pqref.decode_batch(writer.build_batch([ch]))


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["rg0_c2", "rg0_c4", "rg0_c5", "rg1_c4", "rg1_c5"])
def test_harness_levels_nested_fixture(harness, tmp_path, key):
    """checkRead's per-slot sequence (rl, dl, the value when dl == maxDl) through the C level and
    value readers on parquet-mr 1.9.0's nested fixture (phoneNumbers.phone.number / .kind: max
    rep 1, max def 2 / 3) equals the oracle's levels and values."""
    name = "test-file-with-no-column-indexes-1"
    c = next(c for n, c in fixtures.chunk_cases() if n == name and c["key"] == key)
    ch, expected = fixtures.load_chunk(name, c)
    ref = _oracle(ch)
    assert ref.code == 0
    r = parse(run(harness, case_file(tmp_path, raw_chunk(name, c), ch.physical_type, c["num_values"],
                                     type_length=ch.type_length, max_def=c["max_def"], max_rep=c["max_rep"]),
                  "levels"))
    assert r["DECODE"][0] == "0"
    reps, defs, vals = _level_stream(r, sorted(r["pages"]))
    want_d = ref.columns[0]["def_levels"]
    want_r = ref.columns[0]["rep_levels"]
    assert np.array_equal(defs, want_d)
    assert np.array_equal(reps, want_r if want_r is not None else np.zeros_like(defs))
    assert vals == [fmt(v, ch.physical_type) for v in expected]
    assert all(e == (0, "-") for e in r["ends"].values())


@pytest.mark.gpu
@pytest.mark.parametrize("version", [1, 2])
def test_harness_levels_c5_shape(harness, tmp_path, version):
    ch, vals, dl, rl = _c5_chunk(version=version)
    r = parse(run(harness, case_file(tmp_path, thrift_compact.chunk_bytes(ch), abi.INT64, int(dl.size),
                                     max_def=3, max_rep=1), "levels"))
    assert r["DECODE"][0] == "0"
    reps, defs, got = _level_stream(r, sorted(r["pages"]))
    assert np.array_equal(reps, rl) and np.array_equal(defs, dl)
    assert got == [str(int(v)) for v in vals]


def _corrupt_prefix(ch, page, section, cut):
    """Damage a V1 page's level section (0: rl, 1: dl). dl: its 4-byte length prefix shortened by
    `cut` (the stream ends early, the data section starts inside it). rl: its last `cut` bytes
    dropped and the prefix fixed up, so the dl section and the data stay intact behind it."""
    import copy
    bad = copy.deepcopy(ch)
    body = bytearray(bad.pages[page].body)
    at = 0
    if section == 1 and bad.max_rep > 0:
        at = 4 + struct.unpack_from("<i", body, 0)[0]
    n = struct.unpack_from("<i", body, at)[0]
    if section == 0:
        k = max(0, n - cut)
        body = body[:4 + k] + body[4 + n:]
        struct.pack_into("<i", body, 0, k)
    else:
        struct.pack_into("<i", body, at, max(0, n - cut))
    bad.pages[page].body = bytes(body)
    return bad


def _find_error(ch, page, section, phases):
    """A corruption of `page`'s level section for which the oracle fails inside `page` with a
    phase in `phases`."""
    for cut in range(1, 64):
        bad = _corrupt_prefix(ch, page, section, cut)
        ref = _oracle(bad)
        if ref.code and ref.status[1] == page and ref.phase in phases:
            return bad, ref
    pytest.fail("no corruption found")


@pytest.mark.gpu
@pytest.mark.parametrize("section,phases", [(1, (abi.PHASE_DL_READ,)), (0, (abi.PHASE_RL_READ,))])
def test_harness_level_error_at_the_oracles_slot(harness, tmp_path, section, phases):
    """A damaged level section (shortened length prefix) fails at the slot, reader and code where
    the oracle's checkRead fails; the slots and values before it are served, the column's later
    pages are not."""
    ch, vals, dl, rl = _c5_chunk(recs=4000, page_rows=1500)
    bad, ref = _find_error(ch, 1, section, phases)
    code, page, idx = ref.status
    r = parse(run(harness, case_file(tmp_path, thrift_compact.chunk_bytes(bad), abi.INT64, int(dl.size),
                                     max_def=3, max_rep=1), "levels"))
    assert r["DECODE"][:3] == [str(code), abi_exc(code), str(page)]
    assert r["perr"][page][:2] == (code, ref.phase)
    if ref.phase in (abi.PHASE_RL_READ, abi.PHASE_DL_READ):
        assert r["perr"][page][2] == idx
        # slots before the failing one are read, and their values; the failing read raises the code
        got = r["levels"].get(page, [])
        assert [s for s, _, _ in got] == list(range(idx))
        assert r["ends"][page][0] == code
        first = sum(len(pg_levels) for p, pg_levels in r["levels"].items() if p < page)
        assert [d for _, _, d in got] == dl[first:first + idx].tolist()
    else:
        assert r["init"][page][0] == code
    for p in range(page + 1, len(bad.pages)):
        assert r["init"][p][0] == code
    for p in range(page):
        assert r["ends"][p] == (0, "-")


def abi_exc(code):
    import ctypes as C
    L = native.lib()
    L.pqg_java_exception.restype = C.c_char_p
    L.pqg_java_exception.argtypes = [C.c_int]
    e = L.pqg_java_exception(code)
    return e.decode() if e else "-"


@pytest.mark.gpu
def test_harness_error_stays_in_its_column(harness, tmp_path):
    """Two columns in one batch: an invalid dictionary id in column 0 fails column 0's readers at
    that value (and its later pages), column 1 (nested levels + values) reads completely — a
    ColumnReader fails on its own (ColumnReaderBase.java:590-623)."""
    rng = np.random.default_rng(9)
    vals = rng.integers(0, 40, size=30000).astype(np.int64)
    ch0 = writer.write_column_chunk(abi.INT64, vals, abi.RLE_DICTIONARY, page_rows=10000)
    ids, _ = writer.dictionary_encode(vals)
    bad = int(np.argmax(ids >= 35))
    case0 = case_file(tmp_path, thrift_compact.chunk_bytes(ch0, dict_num_values=35), abi.INT64, len(vals), name="c0")
    ch1, v1, dl1, rl1 = _c5_chunk(recs=3000, page_rows=1000)
    case1 = case_file(tmp_path, thrift_compact.chunk_bytes(ch1), abi.INT64, int(dl1.size), max_def=3, max_rep=1,
                      name="c1")
    r = parse(run(harness, case0, "levels", [case1]))
    page, idx = bad // 10000, bad % 10000
    assert r["DECODE"][:4] == [str(abi.ERR_DICT_ID), "java/lang/ArrayIndexOutOfBoundsException", str(page), str(idx)]
    col0 = sorted(p for p, c in r["pagecol"].items() if c == 0)
    col1 = sorted(p for p, c in r["pagecol"].items() if c == 1)
    assert r["perr"][col0[page]] == (abi.ERR_DICT_ID, abi.PHASE_VALUE, idx)
    got = r["values"].get(col0[page], [])
    assert len(got) == idx and all(v == str(int(vals[page * 10000 + k])) for k, v in got)
    assert r["ends"][col0[page]][0] == abi.ERR_DICT_ID
    for p in col0[page + 1:]:
        assert r["init"][p][0] == abi.ERR_DICT_ID
    reps, defs, got1 = _level_stream(r, col1)
    assert np.array_equal(reps, rl1) and np.array_equal(defs, dl1)
    assert got1 == [str(int(v)) for v in v1]
    assert all(r["ends"][p] == (0, "-") for p in col1)


# ---- ParquetReadRouter: a page's runs in one call (pqg_router_read_runs) ----------------------------

def _router_case(tmp_path, w, data, offs, counts):
    p = tmp_path / "router.bin"
    p.write_bytes(b"PQGR" + struct.pack("<iiQ", w, len(counts), len(data)) +
                  np.asarray(offs, dtype="<u8").tobytes() + np.asarray(counts, dtype="<u4").tobytes() + bytes(data))
    return str(p)


def _run_router(router, case, tmp_path):
    outf = tmp_path / "router.out"
    out = subprocess.run([router, case, str(outf)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    f = out.stdout.split()
    return int(f[1]), np.fromfile(str(outf), dtype="<i4")


@pytest.mark.gpu
@pytest.mark.parametrize("w", list(range(33)))
def test_router_batch_matches_oracle(router, tmp_path, w):
    """Many bit-packed runs of one width in one call, each bit-exact with the oracle's
    ParquetReadRouter.readBatch (pqr_router_read_batch) at the same position."""
    from oracle import pqref
    rng = np.random.default_rng(100 + w)
    counts = (rng.integers(1, 64, size=60) * 8).astype(np.uint32)
    gaps = rng.integers(0, 5, size=60)
    offs, pos = [], 0
    for c, g in zip(counts, gaps):
        pos += int(g)
        offs.append(pos)
        pos += int(c) * w // 8
    data = rng.integers(0, 256, size=pos + 3, dtype=np.uint8).tobytes()
    rc, got = _run_router(router, _router_case(tmp_path, w, data, offs, counts), tmp_path)
    assert rc == 0
    want = np.concatenate([pqref.router_read(w, data[o:], int(c))[0] for o, c in zip(offs, counts)])
    assert np.array_equal(got, want)


@pytest.mark.gpu
def test_router_batch_eof_writes_nothing(router, tmp_path):
    """A run whose slice passes the input -> EOF (SingleBufferInputStream.slice) before any unpack."""
    data = bytes(range(100))
    rc, _ = _run_router(router, _router_case(tmp_path, 7, data, [0, 60], [8, 48]), tmp_path)
    assert rc == abi.ERR_EOF


# ---- ParquetReadRouter with its contract: a Spark-style caller loop (pqg_router_read_page) ---------------

REPLAY_SRC = os.path.join(REPO, "tests", "c", "router_replay.c")


@pytest.fixture(scope="module")
def router_replay(tmp_path_factory):
    return _build(tmp_path_factory, REPLAY_SRC, "router_replay")


def _v1_streams(ch):
    """Per V1 page of a chunk: its hybrid sections as (bit_width, n, section bytes, rest of the page
    from the section start): rl / dl level sections (4-byte length prefix) and a dictionary-encoded
    data section (1-byte bit width + ids to the page end)."""
    out = []
    for pg in ch.pages:
        assert pg.version == 1
        b, at = pg.body, 0
        for maxl in (ch.max_rep, ch.max_def):
            if maxl == 0:
                continue
            ln = struct.unpack_from("<i", b, at)[0]
            out.append((writer.width_from_max_int(maxl), pg.num_values, b[at + 4:at + 4 + ln], b[at + 4:]))
            at += 4 + ln
        if pg.encoding in (abi.RLE_DICTIONARY, abi.PLAIN_DICTIONARY) and at < len(b):
            # values count: the slots with d == max_def (the oracle's levels tell; here all for required)
            out.append((b[at], None, b[at + 1:], b[at + 1:]))
    return out


def _replay(router_replay, tmp_path, streams, tail):
    """streams: (w, n, section, page rest). Returns (calls, per-stream (code, decoded), stats)."""
    p = tmp_path / "replay.bin"
    blob = [b"PQGS", struct.pack("<i", len(streams))]
    for w, n, sec, rest in streams:
        s = rest if tail else sec
        blob.append(struct.pack("<iqQQ", w, n, len(sec), len(s)) + bytes(s))
    p.write_bytes(b"".join(blob))
    outf = tmp_path / "replay.out"
    r = subprocess.run([router_replay, str(p), str(outf)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    vals = np.fromfile(str(outf), dtype="<i4")
    calls, res, stats, at = [], [], None, 0
    for ln in r.stdout.splitlines():
        f = ln.split()
        if f[0] == "CALL":
            s, pos, cnt = int(f[1]), int(f[2]), int(f[3])
            calls.append((s, pos, cnt, vals[at:at + cnt]))
            at += cnt
        elif f[0] == "STREAM":
            n = int(f[3])
            res.append((int(f[2]), vals[at:at + n]))
            at += n
        elif f[0] == "STATS":
            stats = (int(f[1]), int(f[2]))
        else:
            pytest.fail(ln)
    return calls, res, stats


def _check_replay(streams, calls, res, stats, strict=True):
    """Every read's buffer on return == the oracle's ParquetReadRouter.readBatch at that position;
    each stream's values == the oracle's RunLengthBitPackingHybridDecoder; one device round trip per
    stream that has bit-packed runs (strict; otherwise at most one: a stream whose first run has the
    bytes, width, count and distance to the stream end of a cached run is served from the cache)."""
    from oracle import pqref
    for s, pos, cnt, got in calls:
        w, _, sec, _ = streams[s]
        want, _ = pqref.router_read(w, bytes(sec[pos:]), cnt)
        assert np.array_equal(got, want), (s, pos, cnt)
    for s, (code, got) in enumerate(res):
        w, n, sec, _ = streams[s]
        want, rc, _, _ = pqref.rle_decode(w, bytes(sec), n)
        assert code == 0 and rc == 0
        assert np.array_equal(got, want), s
    with_packed = len({s for s, _, _, _ in calls})
    assert stats[0] + stats[1] == len(calls)
    assert stats[1] == with_packed if strict else 1 <= stats[1] <= with_packed


@pytest.mark.gpu
@pytest.mark.parametrize("tail", [False, True], ids=["section", "page_rest"])
@pytest.mark.parametrize("zipf", [1.5, 2.0])
def test_router_replay_c2_pages(router_replay, tmp_path, zipf, tail):
    """C2's shape (Zipf runs of ids, w = 10, 20,000-value V1 pages as parquet-mr writes them), read the
    way Spark's readNextGroup reads: header -> ParquetReadRouter.read -> consume currentBuffer at once."""
    from tools import workloads
    ch, _, _ = workloads.make_c2(120_000, a=zipf)
    streams = [(w, pg.num_values, sec, rest) for (w, _, sec, rest), pg in zip(_v1_streams(ch), ch.pages)]
    calls, res, stats = _replay(router_replay, tmp_path, streams, tail)
    assert len(calls) > 10
    _check_replay(streams, calls, res, stats)


@pytest.mark.gpu
@pytest.mark.parametrize("tail", [False, True], ids=["section", "page_rest"])
def test_router_replay_nested_fixture(router_replay, tmp_path, tail):
    """parquet-mr 1.9.0's nested fixture: every rl / dl level section and dictionary id section through
    the caller loop (with page_rest the caller's stream runs on into the page's later sections, which the
    walk parses as if they were runs: those are unpacked and never served)."""
    from oracle import pqref
    name = "test-file-with-no-column-indexes-1"
    streams = []
    for n, c in fixtures.chunk_cases():
        if n != name:
            continue
        ch, _ = fixtures.load_chunk(name, c)
        ref = pqref.decode_batch(writer.build_batch([ch]))
        dl = ref.columns[0]["def_levels"]
        at = 0
        # per page: level streams, then the data stream with n = non-null slots of the page
        for pg in ch.pages:
            ss = _v1_streams(type(ch)(ch.physical_type, ch.max_rep, ch.max_def, ch.type_length, [pg]))
            nn = int((dl[at:at + pg.num_values] == ch.max_def).sum()) if dl is not None else pg.num_values
            streams += [(w, cnt if cnt is not None else nn, sec, rest) for w, cnt, sec, rest in ss]
            at += pg.num_values
    assert len(streams) >= 10
    calls, res, stats = _replay(router_replay, tmp_path, streams, tail)
    # (the fixture's two leaves of one repeated group have equal level sections: the second is a hit)
    _check_replay(streams, calls, res, stats, strict=False)


@pytest.mark.gpu
@pytest.mark.parametrize("w", [1, 2, 3, 7, 8, 10, 13, 16, 20, 24, 31, 32])
def test_router_replay_widths(router_replay, tmp_path, w):
    """Hybrid streams as parquet-mr's encoder writes them (RunLengthBitPackingHybridEncoder: packed runs
    of up to 504 values, RLE runs of repeats), every width class, several streams back to back (the cache
    moves from stream to stream)."""
    rng = np.random.default_rng(500 + w)
    streams = []
    for k in range(4):
        n = int(rng.integers(2000, 9000))
        runs = np.minimum(rng.zipf(1.8, size=n), 300)
        v = np.repeat(rng.integers(0, 1 << min(w, 31), size=runs.size, dtype=np.int64), runs)[:n].astype(np.uint32)
        sec = writer.rle_encode(v, w)
        streams.append((w, n, sec, sec + bytes(rng.integers(0, 256, size=64, dtype=np.uint8))))
    calls, res, stats = _replay(router_replay, tmp_path, streams, True)
    assert calls
    _check_replay(streams, calls, res, stats)


@pytest.mark.gpu
def test_router_page_cache_serves_only_matching_bytes(tmp_path):
    """A cached run is served only for the same width, count, position from the stream end and bytes:
    a different buffer of the same length whose run bytes differ is a miss and decodes its own bytes."""
    from oracle import pqref
    from pqgpu import decoder as D
    dec = D.Decoder(0)
    rng = np.random.default_rng(77)
    v = rng.integers(0, 1 << 9, size=4000).astype(np.uint32)
    sec = np.frombuffer(writer.rle_encode(v, 9), dtype=np.uint8).copy()
    hdr_len = 1 if sec[0] < 0x80 else 2
    count = ((int(sec[0]) & 0x7F) | ((int(sec[1]) & 0x7F) << 7 if hdr_len == 2 else 0)) >> 1
    count *= 8
    got = dec.router_read_page(9, sec, hdr_len, count)
    assert np.array_equal(got, pqref.router_read(9, sec[hdr_len:].tobytes(), count)[0])
    h0, m0 = dec.router_cache_stats()
    other = sec.copy()
    other[hdr_len + 3] ^= 0x5A
    got2 = dec.router_read_page(9, other, hdr_len, count)
    assert np.array_equal(got2, pqref.router_read(9, other[hdr_len:].tobytes(), count)[0])
    h1, m1 = dec.router_cache_stats()
    assert (h1, m1) == (h0, m0 + 1)
    with pytest.raises(native.PqgError) as e:  # the run's bytes past the stream: EOF, nothing written
        dec.router_read_page(9, sec[:hdr_len + 10].copy(), hdr_len, count)
    assert e.value.code == abi.ERR_EOF
