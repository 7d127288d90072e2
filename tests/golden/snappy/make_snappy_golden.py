"""Generate the Snappy golden vectors (tests/golden/snappy/*.bin): inputs compressed by
pyarrow's bundled libsnappy (the same raw block format xerial snappy-java produces for
parquet-mr's SNAPPY pages). Each case is <name>.raw (uncompressed) + <name>.snappy.
Run from the repo root: python tests/golden/snappy/make_snappy_golden.py"""
import os

import numpy as np
import pyarrow as pa

HERE = os.path.dirname(os.path.abspath(__file__))


def cases():
    rng = np.random.default_rng(3)
    yield "text", b"parquet page bytes " * 300 + b"tail"
    yield "random", rng.integers(0, 256, size=5000, dtype=np.uint8).tobytes()          # literals only
    yield "runs", bytes(np.repeat(rng.integers(0, 4, size=400), rng.integers(1, 90, size=400)).astype(np.uint8))
    yield "period3", b"abc" * 2000                                                        # overlapping copies
    yield "longrange", (rng.integers(0, 256, size=20000, dtype=np.uint8).tobytes() * 2)  # offsets > 16 KiB
    yield "int64_page", np.cumsum(rng.integers(-3, 1000, size=8000)).astype(np.int64).tobytes()
    yield "one", b"x"


def main():
    for name, raw in cases():
        comp = pa.compress(raw, codec="snappy", asbytes=True)
        with open(os.path.join(HERE, name + ".raw"), "wb") as f:
            f.write(raw)
        with open(os.path.join(HERE, name + ".snappy"), "wb") as f:
            f.write(comp)
        print(name, len(raw), len(comp))


if __name__ == "__main__":
    main()
