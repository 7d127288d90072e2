"""GZIP page decompression (pqg_gzip_decompress, csrc/pqgpu_gzip.hip): the ORACLE restatement of
RFC 1952 / 1951 (pqr_gzip_decompress, oracle/gzip_ref.c) pinned to Python's zlib on CPU, then the
device decoder against it on zlib streams of every level and strategy (stored, fixed-Huffman and
dynamic blocks), handmade streams (header flags, multi-member pages, codes of 10-15 bits, the single-code
and all-zero code cases, code-length repeats, 32 KiB distances), malformed streams, and pyarrow-written
GZIP parquet fixtures decompressed and decoded end to end on the device.

parquet-mr reads GZIP pages through Hadoop's GzipCodec (CodecFactory.HeapBytesDecompressor,
parquet-hadoop/.../hadoop/CodecFactory.java:155-182: the codec's input stream read for exactly the
page's uncompressed size), a third-party codec absent here: well-formed streams are pinned by zlib
round trips; malformed ones raise in both (ZipException / EOFException there, PQG_ERR_CORRUPT /
PQG_ERR_EOF here). One documented difference between the oracle and the device: the CRC-32 of a member
that ends before the page is complete is checked by the oracle only."""
import gzip
import zlib

import numpy as np
import pytest

from oracle import pqref
from pqgpu import abi
from tools.synth import writer

from fixtures import batch_of, chunk_cases, decompressed_on_host, is_compressed, load_chunk
from helpers import assert_same

# ---- a DEFLATE bit writer for handmade streams ------------------------------------------------------

LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
         227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0] + [k // 2 for k in range(2, 28)]
ORD = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


class Bits:
    def __init__(self):
        self.v, self.n = 0, 0

    def put(self, v, k):  # LSB first
        self.v |= (v & ((1 << k) - 1)) << self.n
        self.n += k

    def code(self, c, k):  # Huffman codes go MSB first
        self.put(int(format(c, f"0{k}b")[::-1], 2) if k else 0, k)

    def align(self):
        self.n = (self.n + 7) // 8 * 8

    def bytes(self):
        return self.v.to_bytes((self.n + 7) // 8, "little")


def canonical(lens):
    """symbol -> (code, length) for code lengths `lens` (RFC 1951 3.2.2)."""
    count = [0] * 16
    for ln in lens:
        count[ln] += 1
    count[0] = 0
    nxt, c = [0] * 16, 0
    for b in range(1, 16):
        c = (c + count[b - 1]) << 1
        nxt[b] = c
    out = {}
    for s, ln in enumerate(lens):
        if ln:
            out[s] = (nxt[ln], ln)
            nxt[ln] += 1
    return out


FIXED_LIT = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
FIXED_DIST = [5] * 30


def _len_sym(n):
    i = max(k for k in range(29) if LBASE[k] <= n)
    return 257 + i, n - LBASE[i], LEXT[i]


def _dist_sym(d):
    i = max(k for k in range(30) if DBASE[k] <= d)
    return i, d - DBASE[i], DEXT[i]


def put_symbols(bw, syms, lit, dist):
    """syms: ints (literal bytes) or (length, distance) pairs, then end-of-block."""
    for s in syms:
        if isinstance(s, tuple):
            ln, d = s
            ls, lx, lb = _len_sym(ln)
            bw.code(*lit[ls])
            bw.put(lx, lb)
            ds, dx, db = _dist_sym(d)
            bw.code(*dist[ds])
            bw.put(dx, db)
        else:
            bw.code(*lit[s])
    bw.code(*lit[256])


def put_dynamic_header(bw, lit_lens, dist_lens, rle=True):
    """HLIT / HDIST / HCLEN and the code lengths, run-length coded with symbols 16 / 17 / 18 when rle."""
    seq = list(lit_lens) + list(dist_lens)
    items, i = [], 0
    while i < len(seq):
        j = i
        while j < len(seq) and seq[j] == seq[i]:
            j += 1
        run = j - i
        if rle and seq[i] == 0 and run >= 11:
            r = min(run, 138)
            items.append((18, r - 11, 7))
        elif rle and seq[i] == 0 and run >= 3:
            r = min(run, 10)
            items.append((17, r - 3, 3))
        elif rle and i > 0 and seq[i] == seq[i - 1] and run >= 3:
            r = min(run, 6)
            items.append((16, r - 3, 2))
        else:
            r = 1
            items.append((seq[i], 0, 0))
        i += r
    cl_lens = [0] * 19
    for s in range(19):  # a complete code-length code: 13 symbols of 4 bits, 6 of 5
        cl_lens[s] = 5 if 10 <= s <= 15 else 4
    clc = canonical(cl_lens)
    bw.put(len(lit_lens) - 257, 5)
    bw.put(len(dist_lens) - 1, 5)
    bw.put(19 - 4, 4)
    for s in ORD:
        bw.put(cl_lens[s], 3)
    for s, x, nb in items:
        bw.code(*clc[s])
        bw.put(x, nb)


def member(deflate, data_for_trailer, flags=0, extra=b"", name=b"", comment=b"", crc=None, isize=None):
    h = bytes([0x1F, 0x8B, 8, flags]) + b"\0\0\0\0" + b"\0\xff"
    if flags & 4:
        h += len(extra).to_bytes(2, "little") + extra
    if flags & 8:
        h += name + b"\0"
    if flags & 16:
        h += comment + b"\0"
    if flags & 2:
        h += (zlib.crc32(h) & 0xFFFF).to_bytes(2, "little")
    c = zlib.crc32(data_for_trailer) if crc is None else crc
    sz = len(data_for_trailer) if isize is None else isize
    return h + deflate + c.to_bytes(4, "little") + sz.to_bytes(4, "little")


def raw_deflate(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY):
    co = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy)
    return co.compress(data) + co.flush()


def expand(syms):
    out = bytearray()
    for s in syms:
        if isinstance(s, tuple):
            ln, d = s
            for _ in range(ln):
                out.append(out[-d])
        else:
            out.append(s)
    return bytes(out)


def _handmade():
    """(stream, expected size, expected bytes)."""
    rng = np.random.default_rng(21)
    cases = []
    # fixed block: literals, overlapping matches of every length symbol and short distances
    syms = [int(b) for b in rng.integers(0, 256, size=40)]
    for ln in (3, 4, 10, 11, 12, 18, 19, 34, 35, 66, 67, 130, 131, 257, 258):
        syms.append((ln, int(rng.integers(1, 30))))
        syms.append(int(rng.integers(0, 256)))
    bw = Bits()
    bw.put(1, 1)
    bw.put(1, 2)
    put_symbols(bw, syms, canonical(FIXED_LIT), canonical(FIXED_DIST))
    bw.align()
    out = expand(syms)
    cases.append((member(bw.bytes(), out), len(out), out))
    # dynamic block with a skewed literal code (lengths 1 .. 15: the 10-15-bit codes take the slow path)
    lit = [0] * 258
    alpha = list(range(65, 65 + 13))
    for k, s in enumerate(alpha):
        lit[s] = k + 1                  # 1 .. 13
    lit[256], lit[257] = 14, 15         # EOB, length 3
    lit[200] = 15
    dist = [0] * 5
    dist[0], dist[4] = 1, 1             # distance 1, distances 5-6
    lc, dc = canonical(lit), canonical(dist)
    syms = []
    for _ in range(3000):
        r = rng.random()
        if r < 0.1 and len(syms) > 8:
            syms.append((3, int(rng.choice([1, 5, 6]))))
        elif r < 0.15:
            syms.append(200)
        else:
            syms.append(alpha[min(int(rng.geometric(0.45)) - 1, 12)])
    bw = Bits()
    bw.put(0, 1)
    bw.put(2, 2)
    put_dynamic_header(bw, lit, dist)
    put_symbols(bw, syms, lc, dc)
    # + an empty dynamic block with a single code (EOB, length 1) and no distance codes, + a stored
    # block, + a final fixed block
    lit1 = [0] * 257
    lit1[256] = 1
    bw.put(0, 1)
    bw.put(2, 2)
    put_dynamic_header(bw, lit1, [0], rle=True)
    bw.code(*canonical(lit1)[256])
    stored = rng.integers(0, 256, size=700, dtype=np.uint8).tobytes()
    bw.put(0, 1)
    bw.put(0, 2)
    bw.align()
    bw.put(len(stored), 16)
    bw.put(~len(stored) & 0xFFFF, 16)
    for b in stored:
        bw.put(b, 8)
    bw.put(1, 1)
    bw.put(1, 2)
    tail = [1, 2, 3, (20, 3)]
    put_symbols(bw, tail, canonical(FIXED_LIT), canonical(FIXED_DIST))
    bw.align()
    out = expand(syms) + stored + expand(tail)
    cases.append((member(bw.bytes(), out), len(out), out))
    # header flags: FEXTRA, FNAME, FCOMMENT, FHCRC
    data = rng.integers(0, 4, size=5000, dtype=np.uint8).tobytes()
    cases.append((member(raw_deflate(data), data, flags=4 | 8 | 16 | 2, extra=b"xy" * 300, name=b"page.bin",
                         comment=b"c" * 99), len(data), data))
    # multi-member page (an empty member in the middle); 32 KiB distances; stored (level 0) member
    far = rng.integers(0, 256, size=20000, dtype=np.uint8).tobytes()
    far = far + bytes(3000) + far[:12000] + far[5000:17000]
    lvl0 = rng.integers(0, 256, size=70000, dtype=np.uint8).tobytes()
    parts = [data, b"", far, lvl0]
    stream = gzip.compress(data) + gzip.compress(b"") + gzip.compress(far, compresslevel=9) + \
        gzip.compress(lvl0, compresslevel=0)
    out = b"".join(parts)
    cases.append((stream, len(out), out))
    # the page completes inside a member: trailing bytes of the member (and garbage after it) unread
    cases.append((gzip.compress(far) + b"garbage", 25000, far[:25000]))
    cases.append((gzip.compress(far, compresslevel=0), 100, far[:100]))
    # empty page; an empty page with no stream at all
    cases.append((gzip.compress(b""), 0, b""))
    cases.append((b"", 0, b""))
    return cases


def _zlib_streams(n_streams=200, seed=4):
    rng = np.random.default_rng(seed)
    strategies = [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FILTERED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE, zlib.Z_FIXED]
    raws, streams = [], []
    for i in range(n_streams):
        n = int(rng.integers(0, 60000))
        kind = i % 5
        if kind == 0:
            raw = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        elif kind == 1:
            raw = bytes(np.repeat(rng.integers(0, 6, size=n // 7 + 1), 7)[:n].astype(np.uint8))
        elif kind == 2:
            raw = np.cumsum(rng.integers(-5, 500, size=n // 8)).astype(np.int64).tobytes()
        elif kind == 3:
            raw = bytes(n)
        else:
            raw = b"".join(f"row-{int(v)};".encode() for v in rng.zipf(1.5, size=n // 8) % 5000)
        level = int(rng.integers(0, 10))
        strat = strategies[(i // 5) % len(strategies)]
        raws.append(raw)
        streams.append(member(raw_deflate(raw, level, strat), raw))
    return raws, streams


def _corrupt_cases():
    """(stream, size, code): malformed in ways both decoders reject the same way."""
    good = gzip.compress(b"hello hello hello hello")
    raw = b"0123456789" * 500
    fx = Bits()
    fx.put(1, 1)
    fx.put(1, 2)
    put_symbols(fx, [65, (3, 2)], canonical(FIXED_LIT), canonical(FIXED_DIST))  # distance 2 > 1 byte written
    fx.align()
    over = Bits()  # over-subscribed literal code
    over.put(1, 1)
    over.put(2, 2)
    put_dynamic_header(over, [1] * 257, [1])
    incomplete = Bits()  # two literal codes of length 2 (incomplete, more than one code)
    incomplete.put(1, 1)
    incomplete.put(2, 2)
    ll = [0] * 257
    ll[65], ll[256] = 2, 2
    put_dynamic_header(incomplete, ll, [1])
    no_eob = Bits()
    no_eob.put(1, 1)
    no_eob.put(2, 2)
    ll = [0] * 257
    ll[65], ll[66] = 1, 1
    put_dynamic_header(no_eob, ll, [1])
    btype3 = Bits()
    btype3.put(1, 1)
    btype3.put(3, 2)
    stored_bad = b"\x01\x05\x00\x00\x00hello"  # NLEN != ~LEN
    E, C = abi.ERR_EOF, abi.ERR_CORRUPT
    return [
        (b"", 5, E),                                         # no stream for a non-empty page
        (good[:6], 23, C),                                   # truncated header
        (b"\x1f\x8c" + good[2:], 23, C),                     # bad magic
        (good[:2] + b"\x07" + good[3:], 23, C),              # CM != 8
        (good[:3] + b"\x20" + good[4:], 23, C),              # reserved flag bit
        (good[:len(good) // 2], 23, C),                      # DEFLATE data cut short
        (good, 24, E),                                       # page longer than the stream
        (member(raw_deflate(raw), raw, isize=7) + good, len(raw) + 23, C),  # wrong ISIZE, non-final member
        (member(fx.bytes(), b"A"), 4, C),                    # distance before the member's start
        (member(over.bytes() + b"\0" * 8, b""), 10, C),
        (member(incomplete.bytes() + b"\0" * 8, b""), 10, C),
        (member(no_eob.bytes() + b"\0" * 8, b""), 10, C),
        (member(btype3.bytes(), b""), 10, C),
        (member(stored_bad, b"hello"), 5, C),
    ]


# ---- CPU: the oracle pinned to zlib ------------------------------------------------------------------

def test_oracle_zlib_round_trips():
    raws, streams = _zlib_streams(100, seed=5)
    for raw, s in zip(raws, streams):
        assert pqref.gzip_decompress(s, len(raw)) == raw
        assert zlib.decompress(s, 31) == raw


def test_oracle_handmade_streams():
    for stream, size, out in _handmade():
        assert pqref.gzip_decompress(stream, size) == out
        if stream:  # zlib agrees with the handmade streams (members read to their end)
            d = zlib.decompressobj(31)
            got = d.decompress(stream)
            while d.eof and d.unused_data[:2] == b"\x1f\x8b":
                rest = d.unused_data
                d = zlib.decompressobj(31)
                got += d.decompress(rest)
            assert got[:size] == out


@pytest.mark.parametrize("k", range(14))
def test_oracle_malformed(k):
    stream, size, code = _corrupt_cases()[k]
    with pytest.raises(ValueError, match=f"error {code}"):
        pqref.gzip_decompress(stream, size)


def test_oracle_checks_crc_of_non_final_members():
    raw = b"abc" * 1000
    bad = member(raw_deflate(raw), raw, crc=zlib.crc32(raw) ^ 1)
    with pytest.raises(ValueError, match=f"error {abi.ERR_CORRUPT}"):
        pqref.gzip_decompress(bad + gzip.compress(b"x"), len(raw) + 1)
    assert pqref.gzip_decompress(bad, len(raw)) == raw  # the completing member's trailer is not read


GZIP_CASES = [(n, c) for n, c in chunk_cases() if c.get("compression") == "GZIP"]


def test_gzip_fixtures_hold_compressed_pages():
    assert len(GZIP_CASES) >= 10
    assert sum(is_compressed(load_chunk(n, c)[0]) for n, c in GZIP_CASES) >= 8


# ---- GPU --------------------------------------------------------------------------------------------

@pytest.fixture(params=["small_pages_wave", "every_page_prepass"])
def prepass(decoder, request):
    """Pages below PQG_DISPATCH_GZIP_PREPASS_MIN (default 16384 output bytes) go to the one-wave
    decoder; with 0 every page takes the token pre-pass (and, for what it hands back, the wave decoder),
    so both paths see every case."""
    if request.param == "every_page_prepass":
        decoder.set_dispatch(abi.DISPATCH_GZIP_PREPASS_MIN, 0)
    yield request.param
    decoder.set_dispatch(abi.DISPATCH_GZIP_PREPASS_MIN, 16384)


def _run(decoder, streams, sizes, skew=False):
    out, offs, status = decoder.gzip_decompress(streams, sizes, skew=skew)
    host = out.cpu().numpy()
    return [host[offs[i]:offs[i] + sizes[i]].tobytes() for i in range(len(streams))], status


@pytest.mark.gpu
@pytest.mark.parametrize("skew", [False, True])
def test_handmade_streams(decoder, skew, prepass):
    cases = _handmade()
    got, status = _run(decoder, [c[0] for c in cases], [c[1] for c in cases], skew=skew)
    assert list(status) == [0] * len(cases)
    for i, (g, (_, _, out)) in enumerate(zip(got, cases)):
        assert g == out, i


@pytest.mark.gpu
@pytest.mark.parametrize("skew", [False, True])
def test_many_zlib_streams(decoder, skew, prepass):
    raws, streams = _zlib_streams()
    got, status = _run(decoder, streams, [len(r) for r in raws], skew=skew)
    assert list(status) == [0] * len(raws)
    assert got == raws


@pytest.mark.gpu
def test_large_pages(decoder):
    """Pages of 160 KB (parquet-mr's int64 pages of 20,000 values, text-like rows) at zlib levels 1, 6
    and 9: dynamic blocks with 259+ literal/length codes, 30 distance codes and 32 KiB distances,
    many blocks per page, tens of thousands of back-references (the token pre-pass's common case)."""
    rng = np.random.default_rng(11)
    raws = []
    for lvl in (1, 6, 9):
        raws.append(np.cumsum(rng.integers(-100, 1000, size=20000)).astype(np.int64).tobytes())
        raws.append(b"".join(f"{int(v)},row-{int(v) % 977};".encode() for v in rng.integers(0, 1 << 30, size=9000)))
    streams = [gzip.compress(r, compresslevel=[1, 1, 6, 6, 9, 9][i]) for i, r in enumerate(raws)]
    got, status = _run(decoder, streams, [len(r) for r in raws])
    assert list(status) == [0] * len(raws)
    assert got == raws


@pytest.mark.gpu
def test_malformed_streams(decoder, prepass):
    cases = _corrupt_cases()
    good = gzip.compress(b"abc")
    streams, sizes = [good], [3]
    for s, n, _ in cases:
        streams += [s, good]
        sizes += [n, 3]
    _, status = _run(decoder, streams, sizes)
    assert all(status[0::2] == 0)
    assert list(status[1::2]) == [c for _, _, c in cases]


@pytest.mark.gpu
def test_crc_of_non_final_members(decoder, prepass):
    """A member that ends before the page has its CRC-32 recomputed on the device (as the oracle and
    Hadoop's GzipCodec stream do): one flipped CRC bit -> CORRUPT; the completing member's trailer is
    not read. Members of 3 KB, 40 KB (stored + compressed) and 0 bytes."""
    rng = np.random.default_rng(5)
    parts = [b"abc" * 1000, rng.integers(0, 40, size=40000, dtype=np.uint8).tobytes(), b""]
    streams, sizes, want = [], [], []
    for raw in parts:
        for lvl in (0, 6):
            for flip in (0, 1, 1 << 31):
                first = member(raw_deflate(raw, level=lvl), raw, crc=zlib.crc32(raw) ^ flip)
                tail = b"tail" * 5000
                streams.append(first + gzip.compress(tail))
                sizes.append(len(raw) + len(tail))
                want.append(abi.ERR_CORRUPT if flip else 0)
                bad_last = member(raw_deflate(raw, level=lvl), raw, crc=zlib.crc32(raw) ^ 1)
                streams.append(gzip.compress(tail) + bad_last)
                sizes.append(len(raw) + len(tail))
                want.append(0)  # the completing member's trailer is not read
    got, status = _run(decoder, streams, sizes)
    assert list(status) == want
    for g, s, n, w in zip(got, streams, sizes, want):
        if w == 0:
            assert g == pqref.gzip_decompress(s, n)


@pytest.mark.gpu
@pytest.mark.parametrize("name,c", GZIP_CASES, ids=[f"{n}:{c['key']}" for n, c in GZIP_CASES])
def test_gzip_fixture_end_to_end(decoder, name, c):
    """File bytes of a GZIP chunk -> GPU decompression into the batch -> GPU decode; the batch equals
    the oracle-decompressed one byte for byte and the values equal pyarrow's."""
    ch, expected = load_chunk(name, c)
    dbatch = decoder.upload_chunks([ch])
    ref_batch = batch_of(ch)
    assert np.array_equal(dbatch.bytes.cpu().numpy(), ref_batch.data)
    cols, st = decoder.decode(dbatch)
    assert_same(cols[0].numpy(), expected, ch.physical_type)


@pytest.mark.gpu
def test_gzip_chunks_with_other_codecs_one_batch(decoder):
    """Synthetic chunks GZIP-compressed like parquet-mr writes them (one member per page; V2: the data
    section), beside LZ4_RAW, SNAPPY and ZSTD chunks, in one upload + decode."""
    from helpers import make, nulls
    rng = np.random.default_rng(3)
    dl = nulls(30000, 0.2, seed=1)
    chunks = [
        writer.gzip_chunk(make(abi.INT64, rng.integers(-9, 9, size=30000), abi.RLE_DICTIONARY, page_rows=7000)),
        writer.gzip_chunk(make(abi.DOUBLE, rng.standard_normal(int(dl.sum())), abi.PLAIN, def_levels=dl, max_def=1,
                               version=2, page_rows=6000), level=1),
        writer.lz4_raw_chunk(make(abi.INT32, rng.integers(-5, 5, size=20000).astype(np.int32), abi.DELTA_BINARY_PACKED)),
        writer.snappy_chunk(make(abi.INT64, np.cumsum(rng.integers(-100, 1000, size=40000)), abi.PLAIN)),
        writer.gzip_chunk(make(abi.BYTE_ARRAY, [bytes([97 + i % 26]) * (i % 13) for i in range(20000)], abi.PLAIN,
                               page_rows=4000), level=9),
        writer.zstd_chunk(make(abi.INT32, rng.integers(0, 1 << 20, size=10000).astype(np.int32), abi.PLAIN)),
    ]
    dbatch = decoder.upload_chunks(chunks)
    ref_batch = writer.build_batch([decompressed_on_host(ch) for ch in chunks])
    assert np.array_equal(dbatch.bytes.cpu().numpy(), ref_batch.data)
    cols, st = decoder.decode(dbatch)
    ref = pqref.decode_batch(ref_batch)
    for i, ch in enumerate(chunks):
        assert_same(cols[i].numpy(), ref.columns[i]["values"], ch.physical_type)
