"""The ZSTD oracle (oracle/zstd_ref.c, RFC 8878 restated) pinned to frames libzstd produced
(tests/golden/zstd/, made by make_zstd_golden.py with pyarrow's bundled libzstd — the library
zstd-jni wraps for parquet-mr's ZSTD pages), XXH64 pinned to the xxhash package, and error cases."""
import glob
import os

import numpy as np
import pytest

from oracle import pqref

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "zstd")
CASES = sorted(os.path.splitext(os.path.basename(p))[0] for p in glob.glob(os.path.join(HERE, "*.zst")))


def load(name):
    return open(os.path.join(HERE, name + ".raw"), "rb").read(), open(os.path.join(HERE, name + ".zst"), "rb").read()


@pytest.mark.parametrize("name", CASES)
def test_golden_frames(name):
    raw, comp = load(name)
    assert pqref.zstd_decompress(comp, len(raw)) == raw


def test_page_reader_takes_the_header_size():
    """BytesInput.from(stream, uncompressedSize): a shorter expected size reads a prefix; a longer one
    runs out of frames (EOF)."""
    raw, comp = load("ints_l3")
    assert pqref.zstd_decompress(comp, 1000) == raw[:1000]
    with pytest.raises(ValueError, match="error 10"):
        pqref.zstd_decompress(comp, len(raw) + 1)


def test_xxh64_matches_xxhash():
    xxhash = pytest.importorskip("xxhash")
    rng = np.random.default_rng(1)
    for n in [0, 1, 3, 4, 7, 8, 31, 32, 33, 100, 1000, 4097]:
        d = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        for seed in (0, 7):
            assert pqref.xxh64(d, seed) == xxhash.xxh64(d, seed=seed).intdigest()


@pytest.mark.parametrize("level", [1, 3, 9, 19, -3])
def test_libzstd_round_trips(level):
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(level + 10)
    for n in [0, 17, 1000, 70000, 300000]:
        for d in (np.cumsum(rng.integers(-50, 900, size=n // 8 + 1)).astype(np.int64).tobytes()[:n],
                  np.minimum(rng.zipf(1.4, size=n), 255).astype(np.uint8).tobytes()):
            c = pa.Codec("zstd", compression_level=level).compress(d, asbytes=True)
            assert pqref.zstd_decompress(c, len(d)) == d


def test_corruption_is_reported():
    raw, comp = load("checksum_l3")
    bad = bytearray(comp)
    bad[-1] ^= 1  # checksum
    with pytest.raises(ValueError, match="error 18"):
        pqref.zstd_decompress(bytes(bad), len(raw))
    bad = bytearray(comp)
    bad[0] ^= 1  # magic
    with pytest.raises(ValueError, match="error 18"):
        pqref.zstd_decompress(bytes(bad), len(raw))
    with pytest.raises(ValueError):
        pqref.zstd_decompress(comp[: len(comp) // 2], len(raw))
    rng = np.random.default_rng(3)
    _, comp = load("zipf_l9")
    for _ in range(200):  # flipped bits anywhere: an error or some output, never a crash
        b = bytearray(comp)
        b[int(rng.integers(4, len(b)))] ^= 1 << int(rng.integers(0, 8))
        try:
            pqref.zstd_decompress(bytes(b), 20000)
        except ValueError:
            pass
