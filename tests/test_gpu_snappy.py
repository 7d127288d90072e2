"""GPU Snappy page decompression (pqg_snappy_decompress, csrc/pqgpu_snappy.hip) vs the committed
golden vectors (pyarrow's libsnappy), the ORACLE decoder on handcrafted blocks (overlapping copies,
copies older than the 32 KiB LDS ring, every literal-length form), malformed blocks, and SNAPPY
parquet fixtures decompressed and decoded end to end on the device."""
import glob
import os

import numpy as np
import pytest

from oracle import pqref
from pqgpu import abi
from tools.synth import writer

from fixtures import batch_of, chunk_cases, decompressed_on_host, is_compressed, load_chunk
from helpers import assert_same

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden", "snappy")


def _varint(n):
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _literal(data):
    n = len(data) - 1
    if n < 60:
        return bytes([n << 2]) + data
    nb = (n.bit_length() + 7) // 8
    return bytes([(59 + nb) << 2]) + n.to_bytes(nb, "little") + data


def _copy(off, length, form):
    if form == 1:
        assert 4 <= length <= 11 and off < 2048
        return bytes([1 | ((length - 4) << 2) | ((off >> 8) << 5), off & 0xFF])
    if form == 2:
        return bytes([2 | ((length - 1) << 2)]) + off.to_bytes(2, "little")
    return bytes([3 | ((length - 1) << 2)]) + off.to_bytes(4, "little")


def _handmade():
    rng = np.random.default_rng(9)
    cases = []
    # overlapping copies (offset < length) of every form, short periods
    body, out = b"", b""
    for period in (1, 2, 3, 5, 7, 16, 63):
        lit = rng.integers(0, 256, size=period, dtype=np.uint8).tobytes()
        body += _literal(lit)
        out += lit
        for form, ln in ((1, 11), (2, 64), (3, 37)):
            body += _copy(period, ln, form)
            for _ in range(ln):
                out += out[-period:-period + 1] if period > 1 else out[-1:]
    cases.append((_varint(len(out)) + body, out))
    # copies older than the LDS ring (offset > 32 KiB) and a literal longer than the 4 KiB segment
    big = rng.integers(0, 256, size=50000, dtype=np.uint8).tobytes()
    body, out = _literal(big), big
    for off in (40000, 32768, 32705, 49999, 12345):
        body += _copy(off, 64, 3)
        out += out[-off:len(out) - off + 64]
    body += _literal(b"end")
    out += b"end"
    cases.append((_varint(len(out)) + body, out))
    # every literal-length form (1..4 extra bytes)
    for n in (60, 61, 300, 70000):
        data = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        cases.append((_varint(n) + _literal(data), data))
    for blob, out in cases:  # the oracle agrees on every handmade block
        assert pqref.snappy_decompress(blob, len(out)) == out
    return cases


def _run(decoder, blocks, sizes, skew=False):
    out, offs, status = decoder.snappy_decompress(blocks, sizes, skew=skew)
    host = out.cpu().numpy()
    return [host[offs[i]:offs[i] + sizes[i]].tobytes() for i in range(len(blocks))], status


def test_golden_vectors(decoder):
    names = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "*.raw")))
    raws = [open(os.path.join(GOLD, n + ".raw"), "rb").read() for n in names]
    comps = [open(os.path.join(GOLD, n + ".snappy"), "rb").read() for n in names]
    got, status = _run(decoder, comps, [len(r) for r in raws])
    assert list(status) == [0] * len(names)
    for n, g, r in zip(names, got, raws):
        assert g == r, n


@pytest.mark.parametrize("skew", [False, True])
def test_handmade_blocks(decoder, skew):
    cases = _handmade()
    got, status = _run(decoder, [c[0] for c in cases], [len(c[1]) for c in cases], skew=skew)
    assert list(status) == [0] * len(cases)
    for i, (g, (_, out)) in enumerate(zip(got, cases)):
        assert g == out, i


@pytest.mark.parametrize("skew", [False, True])
def test_many_pyarrow_blocks(decoder, skew):
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(4)
    raws = []
    for i in range(300):
        n = int(rng.integers(0, 20000))
        kind = i % 3
        if kind == 0:
            raws.append(rng.integers(0, 256, size=n, dtype=np.uint8).tobytes())
        elif kind == 1:
            raws.append(bytes(np.repeat(rng.integers(0, 6, size=n // 7 + 1), 7)[:n].astype(np.uint8)))
        else:
            raws.append(np.cumsum(rng.integers(-5, 500, size=n // 8)).astype(np.int64).tobytes())
    comps = [pa.compress(r, codec="snappy", asbytes=True) for r in raws]
    got, status = _run(decoder, comps, [len(r) for r in raws], skew=skew)
    assert list(status) == [0] * len(raws)
    assert got == raws


@pytest.mark.parametrize("blob,size", [
    (b"\x05\x00a", 5),             # literal shorter than declared
    (b"\x04\x01\x01", 4),          # copy before any output
    (b"\x03\x08abc", 4),           # length differs from the page header's
    (b"\x08\x08abc\x05\x00", 8),   # copy offset 0
    (b"\xff\xff\xff\xff\xff\x01", 1),  # length varint too long
])
def test_malformed_blocks(decoder, blob, size):
    good = b"\x03\x08abc"
    _, status = _run(decoder, [good, blob, good], [3, size, 3])
    assert status[0] == 0 and status[2] == 0
    assert status[1] == abi.ERR_CORRUPT
    with pytest.raises(ValueError):
        pqref.snappy_decompress(blob, size)


SNAPPY_CASES = [(n, c) for n, c in chunk_cases() if c.get("compression") == "SNAPPY"]


def test_snappy_fixtures_hold_compressed_pages():
    assert sum(is_compressed(load_chunk(n, c)[0]) for n, c in SNAPPY_CASES) >= 6


@pytest.mark.parametrize("name,c", SNAPPY_CASES, ids=[f"{n}:{c['key']}" for n, c in SNAPPY_CASES])
def test_snappy_fixture_end_to_end(decoder, name, c):
    """File bytes of a SNAPPY chunk -> GPU decompression into the batch -> GPU decode; the batch
    equals the oracle-decompressed one byte for byte and the values equal pyarrow's."""
    ch, expected = load_chunk(name, c)
    # (a V2 page whose data did not shrink is written with is_compressed = false and stays as is)
    dbatch = decoder.upload_chunks([ch])
    ref_batch = batch_of(ch)
    assert np.array_equal(dbatch.bytes.cpu().numpy(), ref_batch.data)
    cols, st = decoder.decode(dbatch)
    assert_same(cols[0].numpy(), expected, ch.physical_type)
    ref = pqref.decode_batch(ref_batch)
    if c["max_def"] > 0:
        assert np.array_equal(cols[0].def_levels[:ref_batch.column_slots[0]].cpu().numpy(), ref.columns[0]["def_levels"])


def test_snappy_chunks_one_batch(decoder):
    """Synthetic chunks SNAPPY-compressed like parquet-mr writes them (V1 whole body, V2 data
    section), mixed with uncompressed chunks, in one upload + decode."""
    from helpers import make, nulls
    rng = np.random.default_rng(3)
    dl = nulls(30000, 0.2, seed=1)
    chunks = [
        writer.snappy_chunk(make(abi.INT64, rng.integers(-9, 9, size=30000), abi.RLE_DICTIONARY, page_rows=7000)),
        writer.snappy_chunk(make(abi.DOUBLE, rng.standard_normal(int(dl.sum())), abi.PLAIN, def_levels=dl, max_def=1,
                                 version=2, page_rows=6000)),
        make(abi.INT32, rng.integers(-5, 5, size=20000).astype(np.int32), abi.DELTA_BINARY_PACKED),
        writer.snappy_chunk(make(abi.BYTE_ARRAY, [bytes([97 + i % 26]) * (i % 13) for i in range(20000)], abi.PLAIN,
                                 page_rows=4000)),
    ]
    dbatch = decoder.upload_chunks(chunks)
    ref_batch = writer.build_batch([decompressed_on_host(ch) for ch in chunks])
    assert np.array_equal(dbatch.bytes.cpu().numpy(), ref_batch.data)
    cols, st = decoder.decode(dbatch)
    ref = pqref.decode_batch(ref_batch)
    for i, ch in enumerate(chunks):
        assert_same(cols[i].numpy(), ref.columns[i]["values"], ch.physical_type)
