"""Generate the Zstandard golden vectors (tests/golden/zstd/<name>.raw + <name>.zst): inputs compressed
by pyarrow's bundled libzstd (the library zstd-jni wraps for parquet-mr's ZSTD pages), at the level
parquet-mr uses by default (3, ZstandardCodec) and others. Frames with a content checksum are libzstd
frames with the checksum flag set and XXH64 (the `xxhash` package) appended. Run from the repo root:
python tests/golden/zstd/make_zstd_golden.py"""
import os

import numpy as np
import pyarrow as pa
import xxhash

HERE = os.path.dirname(os.path.abspath(__file__))


def zstd(raw, level=3):
    return pa.Codec("zstd", compression_level=level).compress(raw, asbytes=True)


def with_checksum(frame, raw):
    """Set Content_Checksum_Flag (frame header descriptor bit 2) and append XXH64(raw) & 0xFFFFFFFF."""
    b = bytearray(frame)
    assert b[4] & 4 == 0
    b[4] |= 4
    return bytes(b) + (xxhash.xxh64(raw).intdigest() & 0xFFFFFFFF).to_bytes(4, "little")


def cases():
    rng = np.random.default_rng(5)
    ints = np.cumsum(rng.integers(-3, 1000, size=6000)).astype(np.int64).tobytes()
    text = b"parquet page bytes, zstd frames and sequences " * 120
    rnd = rng.integers(0, 256, size=3000, dtype=np.uint8).tobytes()
    zipf = np.minimum(rng.zipf(1.3, size=20000), 255).astype(np.uint8).tobytes()
    dict_ids = np.repeat(rng.integers(0, 1000, size=300), rng.integers(1, 80, size=300)).astype("<u2").tobytes()
    yield "text_l3", text, zstd(text)
    yield "ints_l1", ints, zstd(ints, 1)
    yield "ints_l3", ints, zstd(ints)
    yield "ints_l19", ints, zstd(ints, 19)
    yield "random_l3", rnd, zstd(rnd)                       # incompressible: a raw block
    yield "zipf_l9", zipf, zstd(zipf, 9)                    # Huffman literals, FSE sequence tables
    yield "runs_l3", b"\x07" * 5000, zstd(b"\x07" * 5000)   # RLE
    yield "fast_m5", zipf, zstd(zipf, -5)
    yield "ids_l3", dict_ids, zstd(dict_ids)
    yield "checksum_l3", text, with_checksum(zstd(text), text)
    yield "two_frames", ints + text, zstd(ints) + zstd(text, 9)                      # concatenated frames
    yield "skippable", text, bytes.fromhex("5a2a4d18") + (5).to_bytes(4, "little") + b"skip!" + zstd(text)
    yield "one_byte", b"x", zstd(b"x")
    big = np.cumsum(rng.integers(-100, 1000, size=40000)).astype(np.int64).tobytes()  # 320 KB: 3 blocks
    yield "multi_block_l3", big, zstd(big)


def main():
    for name, raw, comp in cases():
        with open(os.path.join(HERE, name + ".raw"), "wb") as f:
            f.write(raw)
        with open(os.path.join(HERE, name + ".zst"), "wb") as f:
            f.write(comp)
        print(name, len(raw), len(comp))


if __name__ == "__main__":
    main()
