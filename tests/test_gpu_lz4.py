"""LZ4_RAW page decompression (pqg_lz4_raw_decompress, csrc/pqgpu_lz4.hip): the ORACLE restatement
of the LZ4 block format (pqr_lz4_raw_decompress) pinned to pyarrow's liblz4 on CPU, then the device
decoder against it on pyarrow blocks, handmade blocks (overlapping matches, length extensions,
64 KiB offsets, matches older than the 4 KiB LDS ring), malformed blocks, and pyarrow-written LZ4_RAW
parquet fixtures decompressed and decoded end to end on the device.

parquet-mr reads LZ4_RAW pages with Lz4RawDecompressor (parquet-hadoop/.../hadoop/codec/
Lz4RawDecompressor.java:26-50) over aircompressor's Lz4Decompressor, a third-party library absent
here: well-formed blocks are pinned by liblz4 round trips; for malformed blocks both report an error
(aircompressor's MalformedInputException, PQG_ERR_CORRUPT here) — which bytes it names is unpinned."""
import numpy as np
import pytest

from oracle import pqref
from pqgpu import abi
from tools.synth import writer

from fixtures import batch_of, chunk_cases, decompressed_on_host, is_compressed, load_chunk
from helpers import assert_same


def _ext(n):
    """LZ4 length extension bytes for n >= 15 (the nibble holds 15)."""
    n -= 15
    out = bytearray()
    while n >= 255:
        out.append(255)
        n -= 255
    out.append(n)
    return bytes(out)


def _seq(lits, off=None, ml=None):
    """One sequence: literals, then (unless last) a match of ml >= 4 bytes at offset off."""
    ll = len(lits)
    hi = min(ll, 15)
    lo = 0 if ml is None else min(ml - 4, 15)
    body = bytes([(hi << 4) | lo]) + (_ext(ll) if ll >= 15 else b"") + bytes(lits)
    if ml is not None:
        body += off.to_bytes(2, "little") + (_ext(ml - 4) if ml - 4 >= 15 else b"")
    return body


def _handmade():
    """(block, output) pairs covering every form the decoder parses."""
    rng = np.random.default_rng(17)
    cases = []
    # overlapping matches of short periods, long match lengths (extension bytes), literal lengths
    # 0 / 14 / 15 / 270 / 5000
    blk, out = b"", bytearray()
    for period, ml in ((1, 4), (1, 300), (2, 19), (3, 1000), (7, 18), (16, 4096), (63, 70)):
        lit = rng.integers(0, 256, size=period, dtype=np.uint8).tobytes()
        blk += _seq(lit, period, ml)
        out += lit
        for _ in range(ml):
            out.append(out[-period])
    for ll in (0, 14, 15, 270, 5000):
        lit = rng.integers(0, 256, size=ll, dtype=np.uint8).tobytes()
        blk += _seq(lit, 5, 9)
        out += lit
        for _ in range(9):
            out.append(out[-5])
    tail = rng.integers(0, 256, size=40, dtype=np.uint8).tobytes()
    blk += _seq(tail)
    out += tail
    cases.append((blk, bytes(out)))
    # matches far behind (older than the 4 KiB ring, up to 65,535 back)
    base = rng.integers(0, 256, size=70000, dtype=np.uint8).tobytes()
    blk = _seq(base, 65535, 100) + _seq(b"", 4097, 300) + _seq(b"xy", 60000, 5000) + _seq(b"end!!")
    out = bytearray(base)
    for off, ml, lit in ((65535, 100, b""), (4097, 300, b""), (60000, 5000, b"xy")):
        out += lit
        for _ in range(ml):
            out.append(out[-off])
    out += b"end!!"
    cases.append((blk, bytes(out)))
    # empty output (a single 0 token), literals only, one byte
    cases += [(b"\x00", b""), (_seq(b"abc"), b"abc"), (_seq(b"z"), b"z")]
    return cases


def _pyarrow_raws(n_blocks=240, seed=4):
    rng = np.random.default_rng(seed)
    raws = []
    for i in range(n_blocks):
        n = int(rng.integers(0, 30000))
        kind = i % 4
        if kind == 0:
            raws.append(rng.integers(0, 256, size=n, dtype=np.uint8).tobytes())
        elif kind == 1:
            raws.append(bytes(np.repeat(rng.integers(0, 6, size=n // 7 + 1), 7)[:n].astype(np.uint8)))
        elif kind == 2:
            raws.append(np.cumsum(rng.integers(-5, 500, size=n // 8)).astype(np.int64).tobytes())
        else:
            raws.append(bytes(n))
    return raws


MALFORMED = [
    (b"", 0),                        # no input (an empty output is one 0 byte)
    (b"\x50abc", 5),                 # literals past the input
    (b"\x14a\x02\x00", 6),           # match offset past the output (2 > 1)
    (b"\x14a\x00\x00", 6),           # offset 0
    (b"\x10a", 2),                   # output shorter than the header's size
    (b"\x10ab", 1),                  # trailing input after the output is complete
    (b"\x14a\x01\x00\x10b", 3),      # output longer than the header's size
    (b"\xf0\xff\xff", 300),          # literal length extension running off the input
]


# ---- CPU: the oracle pinned to liblz4 -----------------------------------------------------------------

def test_oracle_pyarrow_round_trips():
    pa = pytest.importorskip("pyarrow")
    codec = pa.Codec("lz4_raw")
    for raw in _pyarrow_raws(120, seed=5):
        assert pqref.lz4_raw_decompress(codec.compress(raw, asbytes=True), len(raw)) == raw


def test_oracle_handmade_blocks():
    for blk, out in _handmade():
        assert pqref.lz4_raw_decompress(blk, len(out)) == out
    pa = pytest.importorskip("pyarrow")
    codec = pa.Codec("lz4_raw")
    for blk, out in _handmade():  # liblz4 agrees with the handmade blocks
        assert codec.decompress(blk, decompressed_size=len(out), asbytes=True) == out


@pytest.mark.parametrize("blob,size", MALFORMED)
def test_oracle_malformed(blob, size):
    with pytest.raises(ValueError):
        pqref.lz4_raw_decompress(blob, size)


LZ4_CASES = [(n, c) for n, c in chunk_cases() if c.get("compression") in ("LZ4", "LZ4_RAW")]


def test_lz4_fixtures_hold_compressed_pages():
    assert len(LZ4_CASES) >= 12
    assert sum(is_compressed(load_chunk(n, c)[0]) for n, c in LZ4_CASES) >= 10


# ---- GPU --------------------------------------------------------------------------------------------

def _run(decoder, blocks, sizes, skew=False):
    out, offs, status = decoder.lz4_raw_decompress(blocks, sizes, skew=skew)
    host = out.cpu().numpy()
    return [host[offs[i]:offs[i] + sizes[i]].tobytes() for i in range(len(blocks))], status


@pytest.mark.gpu
@pytest.mark.parametrize("skew", [False, True])
def test_handmade_blocks(decoder, skew):
    cases = _handmade()
    got, status = _run(decoder, [c[0] for c in cases], [len(c[1]) for c in cases], skew=skew)
    assert list(status) == [0] * len(cases)
    for i, (g, (_, out)) in enumerate(zip(got, cases)):
        assert g == out, i


@pytest.mark.gpu
@pytest.mark.parametrize("skew", [False, True])
def test_many_pyarrow_blocks(decoder, skew):
    pa = pytest.importorskip("pyarrow")
    codec = pa.Codec("lz4_raw")
    raws = _pyarrow_raws()
    got, status = _run(decoder, [codec.compress(r, asbytes=True) for r in raws], [len(r) for r in raws], skew=skew)
    assert list(status) == [0] * len(raws)
    assert got == raws


@pytest.mark.gpu
@pytest.mark.parametrize("blob,size", MALFORMED)
def test_malformed_blocks(decoder, blob, size):
    good = _seq(b"abc")
    _, status = _run(decoder, [good, blob, good], [3, size, 3])
    assert status[0] == 0 and status[2] == 0
    assert status[1] == abi.ERR_CORRUPT


@pytest.mark.gpu
@pytest.mark.parametrize("name,c", LZ4_CASES, ids=[f"{n}:{c['key']}" for n, c in LZ4_CASES])
def test_lz4_fixture_end_to_end(decoder, name, c):
    """File bytes of an LZ4_RAW chunk -> GPU decompression into the batch -> GPU decode; the batch
    equals the oracle-decompressed one byte for byte and the values equal pyarrow's."""
    ch, expected = load_chunk(name, c)
    dbatch = decoder.upload_chunks([ch])
    ref_batch = batch_of(ch)
    assert np.array_equal(dbatch.bytes.cpu().numpy(), ref_batch.data)
    cols, st = decoder.decode(dbatch)
    assert_same(cols[0].numpy(), expected, ch.physical_type)


@pytest.mark.gpu
def test_lz4_chunks_with_other_codecs_one_batch(decoder):
    """Synthetic chunks LZ4_RAW-compressed like parquet-mr writes them (V1 whole body, V2 data
    section), beside SNAPPY, ZSTD and uncompressed chunks, in one upload + decode."""
    from helpers import make, nulls
    rng = np.random.default_rng(3)
    dl = nulls(30000, 0.2, seed=1)
    chunks = [
        writer.lz4_raw_chunk(make(abi.INT64, rng.integers(-9, 9, size=30000), abi.RLE_DICTIONARY, page_rows=7000)),
        writer.lz4_raw_chunk(make(abi.DOUBLE, rng.standard_normal(int(dl.sum())), abi.PLAIN, def_levels=dl, max_def=1,
                                  version=2, page_rows=6000)),
        writer.snappy_chunk(make(abi.INT32, rng.integers(-5, 5, size=20000).astype(np.int32), abi.DELTA_BINARY_PACKED)),
        writer.zstd_chunk(make(abi.INT64, np.cumsum(rng.integers(-100, 1000, size=40000)), abi.PLAIN)),
        writer.lz4_raw_chunk(make(abi.BYTE_ARRAY, [bytes([97 + i % 26]) * (i % 13) for i in range(20000)], abi.PLAIN,
                                  page_rows=4000)),
    ]
    dbatch = decoder.upload_chunks(chunks)
    ref_batch = writer.build_batch([decompressed_on_host(ch) for ch in chunks])
    assert np.array_equal(dbatch.bytes.cpu().numpy(), ref_batch.data)
    cols, st = decoder.decode(dbatch)
    ref = pqref.decode_batch(ref_batch)
    for i, ch in enumerate(chunks):
        assert_same(cols[i].numpy(), ref.columns[i]["values"], ch.physical_type)
