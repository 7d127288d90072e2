"""ORACLE Snappy decoder (oracle/pqref.c pqr_snappy_decompress) pinned to the committed golden
vectors (compressed by pyarrow's libsnappy; tests/golden/snappy/make_snappy_golden.py) and to
fresh pyarrow round trips; malformed blocks are errors."""
import glob
import os

import numpy as np
import pytest

from oracle import pqref

GOLD = os.path.join(os.path.dirname(__file__), "golden", "snappy")
CASES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "*.raw")))


@pytest.mark.parametrize("name", CASES)
def test_golden(name):
    raw = open(os.path.join(GOLD, name + ".raw"), "rb").read()
    comp = open(os.path.join(GOLD, name + ".snappy"), "rb").read()
    assert pqref.snappy_decompress(comp, len(raw)) == raw


def test_pyarrow_round_trips():
    pa = pytest.importorskip("pyarrow")
    rng = np.random.default_rng(5)
    for n in [0, 1, 7, 64, 65, 1000, 70000]:
        for kind in range(3):
            if kind == 0:
                raw = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
            elif kind == 1:
                raw = bytes(np.repeat(rng.integers(0, 3, size=n // 5 + 1), 5)[:n].astype(np.uint8))
            else:
                raw = (b"0123456789abcdef" * (n // 16 + 1))[:n]
            comp = pa.compress(raw, codec="snappy", asbytes=True)
            assert pqref.snappy_decompress(comp, n) == raw


@pytest.mark.parametrize("blob,size", [
    (b"", 0),                      # no length varint
    (b"\x05\x00a", 5),             # literal shorter than declared
    (b"\x04\x01\x01", 4),          # copy before any output (offset > position)
    (b"\x03\x08abc", 4),           # declared length differs from the header's uncompressed size
    (b"\x08\x08abc\x05\x00", 8),   # copy with offset 0
])
def test_malformed(blob, size):
    with pytest.raises(ValueError):
        pqref.snappy_decompress(blob, size)
