"""GPU ZSTD page decompression (pqg_zstd_decompress, csrc/pqgpu_zstd.hip) vs the committed golden
frames (libzstd, tests/golden/zstd/), the ORACLE (oracle/zstd_ref.c) on libzstd frames of every
level / block shape, malformed and bit-flipped frames (the device and the oracle agree on success,
failure and output), and ZSTD parquet fixtures decompressed and decoded end to end on the device."""
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
GOLD = os.path.join(os.path.dirname(__file__), "golden", "zstd")


def _run(decoder, frames, sizes):
    out, offs, status, _ = decoder.zstd_decompress(frames, sizes)
    host = out.cpu().numpy()
    return [host[offs[i]:offs[i] + sizes[i]].tobytes() for i in range(len(frames))], status


def _oracle(frame, size):
    try:
        return 0, pqref.zstd_decompress(frame, size)
    except ValueError as e:
        return int(str(e).split("error ")[1].split()[0].rstrip(")")), None


def test_golden_frames(decoder):
    names = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "*.zst")))
    raws = [open(os.path.join(GOLD, n + ".raw"), "rb").read() for n in names]
    comps = [open(os.path.join(GOLD, n + ".zst"), "rb").read() for n in names]
    got, status = _run(decoder, comps, [len(r) for r in raws])
    assert list(status) == [0] * len(names)
    for n, g, r in zip(names, got, raws):
        assert g == r, n


@pytest.mark.parametrize("level", [1, 3, 9, 19, -5])
def test_libzstd_frames(decoder, level):
    """Many frames at once: raw / RLE / compressed blocks, predefined / RLE / FSE / repeat tables,
    1- and 4-stream literals, multi-block frames with matches reaching into earlier blocks."""
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(100 + level)
    raws = []
    for i in range(120):
        n = int(rng.choice([0, 1, 40, 700, 5000, 40000, 140000, 400000])) if i % 5 else int(rng.integers(0, 3000))
        kind = i % 5
        if kind == 0:
            raws.append(rng.integers(0, 256, size=n, dtype=np.uint8).tobytes())
        elif kind == 1:
            raws.append(bytes(np.repeat(rng.integers(0, 6, size=n // 7 + 1), 7)[:n].astype(np.uint8)))
        elif kind == 2:
            raws.append(np.cumsum(rng.integers(-5, 500, size=n // 8 + 1)).astype(np.int64).tobytes()[:n])
        elif kind == 3:
            raws.append(np.minimum(rng.zipf(1.3, size=n), 255).astype(np.uint8).tobytes())
        else:
            words = [bytes(rng.integers(97, 123, size=int(rng.integers(2, 12)), dtype=np.uint8)) for _ in range(50)]
            raws.append(b"".join(words[int(j)] for j in rng.integers(0, 50, size=n // 6 + 1))[:n])
    codec = pa.Codec("zstd", compression_level=level)
    comps = [codec.compress(r, asbytes=True) for r in raws]
    got, status = _run(decoder, comps, [len(r) for r in raws])
    bad = [(i, int(status[i]), len(raws[i]), len(comps[i]), i % 5) for i in range(len(raws)) if status[i]]
    assert not bad, bad
    for i, (g, r) in enumerate(zip(got, raws)):
        assert g == r, (i, len(r))


def test_header_size_and_concatenated_frames(decoder):
    """The page reader takes the header's uncompressed size: a shorter size keeps a prefix, a
    longer one runs out of frames (EOF); concatenated and skippable frames decode in order."""
    pa = pytest.importorskip("pyarrow")
    raw = open(os.path.join(GOLD, "ints_l3.raw"), "rb").read()
    comp = open(os.path.join(GOLD, "ints_l3.zst"), "rb").read()
    a = np.arange(3000, dtype=np.int32).tobytes()
    ca = pa.Codec("zstd", compression_level=5).compress(a, asbytes=True)
    skip = (0x184D2A53).to_bytes(4, "little") + (9).to_bytes(4, "little") + bytes(9)
    frames = [comp, comp, ca + skip + comp]
    sizes = [1000, len(raw) + 1, len(a) + len(raw)]
    got, status = _run(decoder, frames, sizes)
    assert status[0] == 0 and got[0] == raw[:1000]
    assert status[1] == abi.ERR_EOF
    assert status[2] == 0 and got[2] == a + raw
    assert _oracle(frames[1], sizes[1])[0] == abi.ERR_EOF
    assert _oracle(frames[2], sizes[2]) == (0, a + raw)


def test_malformed_frames(decoder):
    raw = open(os.path.join(GOLD, "checksum_l3.raw"), "rb").read()
    comp = open(os.path.join(GOLD, "checksum_l3.zst"), "rb").read()
    bad_sum, bad_magic = bytearray(comp), bytearray(comp)
    bad_sum[-1] ^= 1
    bad_magic[0] ^= 1
    frames = [comp, bytes(bad_sum), bytes(bad_magic), comp[: len(comp) // 2], b"", comp]
    got, status = _run(decoder, frames, [len(raw)] * len(frames))
    assert status[0] == 0 and status[5] == 0 and got[0] == raw and got[5] == raw
    assert status[1] == abi.ERR_CORRUPT and status[2] == abi.ERR_CORRUPT
    assert status[3] in (abi.ERR_CORRUPT, abi.ERR_EOF) and status[4] in (abi.ERR_CORRUPT, abi.ERR_EOF)
    for i in (1, 2, 3, 4):
        assert _oracle(frames[i], len(raw))[0] == status[i], i


def test_bit_flips_agree_with_oracle(decoder):
    """Flipped bits anywhere in libzstd frames: the device never faults or hangs, and reports what
    the oracle reports (same error class, or success with the same bytes)."""
    rng = np.random.default_rng(11)
    names = ["zipf_l9", "ints_l3", "text_l3", "multi_block_l3"]
    frames, sizes = [], []
    for n in names:
        raw = open(os.path.join(GOLD, n + ".raw"), "rb").read()
        comp = open(os.path.join(GOLD, n + ".zst"), "rb").read()
        for _ in range(150):
            b = bytearray(comp)
            for _ in range(int(rng.integers(1, 3))):
                b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
            frames.append(bytes(b))
            sizes.append(len(raw))
    got, status = _run(decoder, frames, sizes)
    mism = []
    for i, (f, s) in enumerate(zip(frames, sizes)):
        code, val = _oracle(f, s)
        if (code == 0) != (status[i] == 0) or (code == 0 and got[i] != val):
            mism.append((i, code, int(status[i])))
    assert not mism, mism[:10]


ZSTD_CASES = [(n, c) for n, c in chunk_cases() if c.get("compression") == "ZSTD"]


def test_zstd_fixtures_hold_compressed_pages():
    assert sum(is_compressed(load_chunk(n, c)[0]) for n, c in ZSTD_CASES) >= 6


@pytest.mark.parametrize("name,c", ZSTD_CASES, ids=[f"{n}:{c['key']}" for n, c in ZSTD_CASES])
def test_zstd_fixture_end_to_end(decoder, name, c):
    """File bytes of a ZSTD chunk (pyarrow-written) -> GPU decompression into the batch -> GPU
    decode; the batch equals the oracle-decompressed one byte for byte, the values equal pyarrow's."""
    ch, expected = load_chunk(name, c)
    dbatch = decoder.upload_chunks([ch])
    ref_batch = batch_of(ch)
    assert np.array_equal(dbatch.bytes.cpu().numpy(), ref_batch.data)
    cols, st = decoder.decode(dbatch)
    assert_same(cols[0].numpy(), expected, ch.physical_type)


def test_mixed_codecs_one_batch(decoder):
    """ZSTD, SNAPPY and uncompressed chunks (V1 whole body, V2 data section) in one upload + decode."""
    from helpers import make, nulls
    rng = np.random.default_rng(5)
    dl = nulls(30000, 0.2, seed=2)
    chunks = [
        writer.zstd_chunk(make(abi.INT64, rng.integers(-9, 9, size=30000), abi.RLE_DICTIONARY, page_rows=7000)),
        writer.zstd_chunk(make(abi.DOUBLE, rng.standard_normal(int(dl.sum())), abi.PLAIN, def_levels=dl, max_def=1,
                               version=2, page_rows=6000), level=9),
        writer.snappy_chunk(make(abi.INT32, rng.integers(-5, 5, size=20000).astype(np.int32), abi.DELTA_BINARY_PACKED)),
        make(abi.FLOAT, rng.standard_normal(5000).astype(np.float32), abi.PLAIN),
        writer.zstd_chunk(make(abi.BYTE_ARRAY, [bytes([97 + i % 26]) * (i % 13) for i in range(20000)], abi.PLAIN,
                               page_rows=4000), level=1),
    ]
    dbatch = decoder.upload_chunks(chunks)
    ref_batch = writer.build_batch([decompressed_on_host(ch) for ch in chunks])
    assert np.array_equal(dbatch.bytes.cpu().numpy(), ref_batch.data)
    cols, st = decoder.decode(dbatch)
    ref = pqref.decode_batch(ref_batch)
    for i, ch in enumerate(chunks):
        assert_same(cols[i].numpy(), ref.columns[i]["values"], ch.physical_type)
