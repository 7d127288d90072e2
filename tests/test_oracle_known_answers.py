"""Known-answer tests transcribed from the reference's own unit tests.

Each test names the reference test it restates. The writer (libpqwriter) restates
parquet-mr's encoders and is checked against the exact bytes the reference tests
assert; the oracle (oracle/pqref.c) decodes them value for value.
"""
import numpy as np
import pytest

from javarandom import JavaRandom
from oracle import pqref
from pqgpu import abi
from tools.synth import writer


def uvarint(v):
    out = bytearray()
    while v & ~0x7F:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def pack_lsb(values, w):
    """Independent LSB-first packer (numpy bit arithmetic)."""
    bits = np.zeros(len(values) * w, dtype=np.uint8)
    for i, v in enumerate(values):
        for k in range(w):
            bits[i * w + k] = (int(v) >> k) & 1
    return np.packbits(bits, bitorder="little").tobytes()


# ---- TestRunLengthBitPackingHybridEncoder (rle/TestRunLengthBitPackingHybridEncoder.java) ----------------------

def test_rle_only():  # :45-69
    enc = writer.rle_encode([4] * 100 + [5] * 100, 3)
    assert enc == uvarint(200) + bytes([4]) + uvarint(200) + bytes([5])
    vals, rc, _, cons = pqref.rle_decode(3, enc, 200)
    assert rc == 0 and cons == len(enc)
    assert list(vals) == [4] * 100 + [5] * 100


def test_repeated_zeros():  # :71-91
    enc = writer.rle_encode([0] * 10, 3)
    assert enc == uvarint(20) + bytes([0])


def test_bit_width_zero():  # :93-107
    enc = writer.rle_encode([0] * 10, 0)
    assert enc == uvarint(20)
    vals, rc, _, _ = pqref.rle_decode(0, enc, 10)
    assert rc == 0 and list(vals) == [0] * 10


def test_bit_packing_only():  # :109-129
    vals = [i % 3 for i in range(100)]
    enc = writer.rle_encode(vals, 3)
    assert enc == uvarint(27) + pack_lsb(vals + [0] * 4, 3)
    dec, rc, _, _ = pqref.rle_decode(3, enc, 100)
    assert rc == 0 and list(dec) == vals


def test_bit_packing_overflow():  # :131-161, 504-value cap -> headers 127 and 125
    vals = [i % 3 for i in range(1000)]
    enc = writer.rle_encode(vals, 3)
    assert enc == uvarint(127) + pack_lsb(vals[:504], 3) + uvarint(125) + pack_lsb(vals[504:], 3)
    dec, rc, _, _ = pqref.rle_decode(3, enc, 1000)
    assert rc == 0 and list(dec) == vals


def test_transition_from_bit_packing_to_rle():  # :163-199
    vals = [0, 1, 0, 1, 0, 2, 2, 2] + [2] * 100
    enc = writer.rle_encode(vals, 3)
    assert enc == uvarint(3) + pack_lsb([0, 1, 0, 1, 0, 2, 2, 2], 3) + uvarint(200) + bytes([2])
    dec, rc, _, _ = pqref.rle_decode(3, enc, len(vals))
    assert rc == 0 and list(dec) == vals


def test_padding_zeros_on_unfinished_bit_packed_runs():  # :201-218
    vals = list(range(1, 10))
    enc = writer.rle_encode(vals, 5)
    assert enc == uvarint(5) + pack_lsb(vals + [0] * 7, 5)


def test_switching_modes():  # :220-285, w = 9 -> 2-byte RLE values
    vals = [17] * 25 + [7] * 7 + [8, 9, 10] + [6] * 25 + [5] * 8
    enc = writer.rle_encode(vals, 9)
    exp = (uvarint(50) + (17).to_bytes(2, "little") + uvarint(5) + pack_lsb([7] * 7 + [8, 9, 10] + [6] * 6, 9) +
           uvarint(38) + (6).to_bytes(2, "little") + uvarint(16) + (5).to_bytes(2, "little"))
    assert enc == exp
    dec, rc, _, _ = pqref.rle_decode(9, enc, len(vals))
    assert rc == 0 and list(dec) == vals


def test_group_boundary():  # :287-300: 3 values of one literal group in 2 bytes, rest zero-filled
    data = bytes([(1 << 1) | 1, (1 << 0) | (2 << 2) | (3 << 4)])
    dec, rc, _, cons = pqref.rle_decode(2, data, 8)
    assert rc == 0 and list(dec[:3]) == [1, 2, 3] and list(dec[3:]) == [0] * 5
    assert cons == 2


# ---- RunLengthBitPackingHybridIntegrationTest (:30-85) ------------------------------------------------------------

@pytest.mark.parametrize("w", range(0, 33))
def test_rle_integration_all_widths(w):
    mod = 1 << w
    vals = [i % mod for i in range(100)] + [77 % mod] * 100 + [88 % mod] * 100
    for i in range(1000):
        vals += [i % mod] * 3
    vals += [17 % mod] * 1000
    vals = np.array(vals, dtype=np.uint64).astype(np.uint32).view(np.int32)
    enc = writer.rle_encode(vals, w)
    dec, rc, _, _ = pqref.rle_decode(w, enc, len(vals))
    assert rc == 0
    assert np.array_equal(dec, vals)


# ---- decoder error semantics (RunLengthBitPackingHybridDecoder.java:55, :81) --------------------------------------

def test_rle_read_past_end():
    enc = writer.rle_encode([1] * 20, 2)
    dec, rc, idx, _ = pqref.rle_decode(2, enc, 25)
    assert rc == abi.ERR_RLE_PAST_END and idx == 20


def test_rle_bad_bit_width():
    _, rc, idx, _ = pqref.rle_decode(33, b"\x02\x01", 1)
    assert rc == abi.ERR_BIT_WIDTH and idx == 0


def test_rle_truncated_value_is_eof():
    _, rc, idx, _ = pqref.rle_decode(16, uvarint(40) + b"\x01", 5)  # 2 value bytes needed, 1 present
    assert rc == abi.ERR_EOF and idx == 0


def test_rle_zero_count_run_repeats_forever():
    # header 0 -> RLE run of 0: Java decrements currentCount below 0 and keeps returning the value
    dec, rc, _, _ = pqref.rle_decode(4, bytes([0, 9]), 50)
    assert rc == 0 and list(dec) == [9] * 50


def test_rle_empty_packed_run():
    _, rc, idx, _ = pqref.rle_decode(4, bytes([1, 0, 0]), 1)
    assert rc == abi.ERR_EMPTY_PACKED_RUN and idx == 0


def test_rle_unmasked_value():
    # readIntLittleEndianPaddedOnBitWidth does not mask to w: w = 3 reads one byte, 0xFF stays 255
    dec, rc, _, _ = pqref.rle_decode(3, uvarint(16) + b"\xff", 8)
    assert rc == 0 and list(dec) == [255] * 8


# ---- bit packers (TestByteBitPacking.java, LSB-first LITTLE_ENDIAN packers) -----------------------------------

@pytest.mark.parametrize("w", range(0, 33))
def test_unpack8_int_all_widths(w):
    rng = np.random.default_rng(w)
    vals = rng.integers(0, 1 << w, size=8, dtype=np.uint64) if w else np.zeros(8, np.uint64)
    packed = pack_lsb([int(v) for v in vals], w)
    got = pqref.unpack8_int(w, packed.ljust(max(w, 1), b"\0"))
    assert np.array_equal(got.astype(np.uint32), vals.astype(np.uint32))


@pytest.mark.parametrize("w", range(0, 65))
def test_unpack8_long_all_widths(w):
    rng = np.random.default_rng(100 + w)
    vals = [int(x) for x in (rng.integers(0, 1 << min(w, 62), size=8, dtype=np.uint64))]
    if w > 62:
        vals = [v | ((i & 1) << (w - 1)) for i, v in enumerate(vals)]
    packed = pack_lsb(vals, w)
    got = pqref.unpack8_long(w, packed.ljust(max(w, 1), b"\0"))
    assert [int(x) & ((1 << 64) - 1) for x in got.astype(np.uint64)] == vals


@pytest.mark.parametrize("w", [1, 3, 8, 10, 17, 31, 32])
def test_router_read_batch(w):
    """ParquetReadRouter.readBatch: per 8 values unpack8Values over w bytes."""
    rng = np.random.default_rng(w)
    vals = [int(v) for v in rng.integers(0, 1 << w, size=128, dtype=np.uint64)]
    packed = pack_lsb(vals, w)
    got, consumed = pqref.router_read(w, packed, 128)
    assert consumed == 128 * w // 8
    assert [int(x) & 0xFFFFFFFF for x in got] == vals
    with pytest.raises(EOFError):
        pqref.router_read(w, packed[:-1], 128)


# ---- DeltaBinaryPackingValuesWriterFor{Long,Integer}Test (delta/*Test.java:57-227) ------------------------------

BLOCK, MB = 128, 4


def _long_cases():
    def rand_longs(n):
        r = JavaRandom(0)
        return [r.nextLong() for _ in range(n)]

    def neg():
        r = JavaRandom(0)
        return [10 - (i * 32 - r.nextInt(6)) for i in range(BLOCK)]

    def unaligned():
        r = JavaRandom(0)
        return [r.nextInt(20) - 10 for _ in range(5 * BLOCK + 3)]

    return {
        "aligned_with_block": rand_longs(5 * BLOCK),                    # :57-65
        "block_not_fully_written": rand_longs(BLOCK - 3),              # :67-74
        "miniblock_not_fully_written": rand_longs(BLOCK // MB - 3),    # :76-83
        "negative_deltas": neg(),                                      # :85-92
        "deltas_same": [i * 32 for i in range(BLOCK)] + [0] * BLOCK,   # :94-101
        "values_same": [3] * BLOCK + [0] * BLOCK,                      # :103-110
        "delta0_each_block": [(i - 1) // BLOCK if i > 0 else 0 for i in range(5 * BLOCK + 1)],  # :112-119 (Java / truncates)
        "not_aligned_with_block": unaligned(),                          # :121-128
        "max_min": [(-2**63 if i % 2 == 0 else 2**63 - 1) for i in range(10)],  # :130-141
    }


@pytest.mark.parametrize("case", list(_long_cases().keys()))
def test_delta_long_round_trip(case):
    data = np.array(_long_cases()[case], dtype=np.int64)
    enc = writer.delta_encode(data, abi.INT64, BLOCK, MB)
    got, consumed = pqref.delta_decode(enc)
    assert consumed == len(enc)  # shouldReturnCorrectOffsetAfterInitialization (:143-177)
    assert np.array_equal(got, data)


def _int_cases():
    def rand_ints(n):
        r = JavaRandom(0)
        return [r.nextInt() for _ in range(n)]

    neg = JavaRandom(0)
    un = JavaRandom(0)
    return {
        "aligned_with_block": rand_ints(5 * BLOCK),
        "block_not_fully_written": rand_ints(BLOCK - 3),
        "miniblock_not_fully_written": rand_ints(BLOCK // MB - 3),
        "negative_deltas": [10 - (i * 32 - neg.nextInt(6)) for i in range(BLOCK)],
        "values_same": [3] * BLOCK + [0] * BLOCK,
        "not_aligned_with_block": [un.nextInt(20) - 10 for _ in range(5 * BLOCK + 3)],
        "max_min": [(-2**31 if i % 2 == 0 else 2**31 - 1) for i in range(10)],
    }


@pytest.mark.parametrize("case", list(_int_cases().keys()))
def test_delta_int_round_trip(case):
    data = np.array(_int_cases()[case], dtype=np.int32)
    enc = writer.delta_encode(data, abi.INT32, BLOCK, MB)
    got, consumed = pqref.delta_decode(enc)
    assert consumed == len(enc)
    assert np.array_equal(got.astype(np.int64).astype(np.int32), data)  # readInteger = (int) readLong


def test_delta_read_past_end():  # shouldThrowExceptionWhenReadMoreThanWritten (:179-191)
    data = np.arange(5 * BLOCK + 1, dtype=np.int64) * 32
    ch = writer.write_column_chunk(abi.INT64, data, abi.DELTA_BINARY_PACKED, page_rows=10**9)
    ch.pages[0].num_values = len(data) + 1
    res = pqref.decode_batch(writer.build_batch([ch]))
    assert res.code == abi.ERR_DELTA_PAST_END and res.status == (abi.ERR_DELTA_PAST_END, 0, len(data))


def test_delta_minblock_not_multiple_of_8():  # miniBlockSizeShouldBeMultipleOf8 (:52-55): reader side
    enc = uvarint(1281) + uvarint(4) + uvarint(3) + b"\x00"
    code, _ = pqref.delta_decode(enc)
    assert code == abi.ERR_DELTA_CONFIG


# ---- TestDictionary.testLongDictionary (:285-317) and testZeroValues (:659-679) ---------------------------------

def test_long_dictionary_two_pages():
    v1 = [i % 50 for i in range(1000)]
    v2 = [i % 50 for i in range(2000, 0, -1)]
    ch = writer.write_column_chunk(abi.INT64, np.array(v1 + v2, dtype=np.int64), abi.PLAIN_DICTIONARY, page_rows=1000)
    assert ch.dict_num_values == 50
    res = pqref.decode_batch(writer.build_batch([ch]))
    assert res.code == 0 and list(res.columns[0]["values"]) == v1 + v2


def test_dictionary_empty_data_section():
    """All-null page: empty data section, nothing read -> no error (testZeroValues)."""
    dl = np.zeros(100, dtype=np.uint8)
    ch = writer.write_column_chunk(abi.INT32, np.zeros(0, dtype=np.int32), abi.PLAIN_DICTIONARY, def_levels=dl,
                                   max_def=1)
    ch.dict_page = (34).to_bytes(4, "little")
    ch.dict_num_values = 1
    # the reader gets a data section of 0 bytes
    res = pqref.decode_batch(writer.build_batch([ch]))
    assert res.code == 0 and res.columns[0]["n_values"] == 0


def test_dictionary_page_encoding_must_be_plain():  # PlainValuesDictionary.java:49-52
    ch = writer.write_column_chunk(abi.INT64, np.arange(10, dtype=np.int64), abi.RLE_DICTIONARY)
    ch.dict_encoding = abi.RLE
    res = pqref.decode_batch(writer.build_batch([ch]))
    assert res.code == abi.ERR_DICT_ENCODING


# ---- TestDeltaLengthByteArray / TestDeltaByteArray (deltalengthbytearray/, deltastrings/) ------------------------

def _decode_bytes(enc, values, ptype=abi.BYTE_ARRAY, **kw):
    ch = writer.write_column_chunk(ptype, values, enc, **kw)
    return pqref.decode_batch(writer.build_batch([ch]))


def test_dlba_serialization():  # TestDeltaLengthByteArray.testSerialization / testLengths
    vals = [b"parquet", b"hadoop", b"mapreduce"]
    data = writer.dlba_encode(vals)
    lens, consumed = pqref.delta_decode(data)
    assert list(lens) == [7, 6, 9] and data[consumed:] == b"parquethadoopmapreduce"
    res = _decode_bytes(abi.DELTA_LENGTH_BYTE_ARRAY, vals)
    assert res.code == 0 and res.columns[0]["values"] == vals


def test_dba_serialization_and_lengths():  # TestDeltaByteArray.testSerialization / testLengths (:35-90)
    vals = [b"parquet-mr", b"parquet", b"parquet-format"]
    data = writer.dba_encode(vals)
    prefix, c1 = pqref.delta_decode(data)
    assert list(prefix) == [0, 7, 7]
    suffix, _ = pqref.delta_decode(data[c1:])
    assert list(suffix) == [10, 0, 7]
    res = _decode_bytes(abi.DELTA_BYTE_ARRAY, vals)
    assert res.code == 0 and res.columns[0]["values"] == vals


@pytest.mark.parametrize("enc", [abi.DELTA_LENGTH_BYTE_ARRAY, abi.DELTA_BYTE_ARRAY, abi.PLAIN])
def test_binary_random_strings(enc):  # testRandomStrings: 10,000 strings of <= 32 chars
    rng = np.random.default_rng(10)
    vals = [bytes(rng.integers(97, 123, size=rng.integers(0, 33), dtype=np.uint8)) for _ in range(10000)]
    vals.sort()
    res = _decode_bytes(enc, vals, page_rows=3000)
    assert res.code == 0 and res.columns[0]["values"] == vals


def test_dba_prefix_longer_than_previous_fails():
    """arraycopy(previous, 0, out, 0, prefixLength) with prefixLength > previous.length (:70-73)."""
    data = writer.delta_encode(np.array([3], dtype=np.int32), abi.INT32) + writer.dlba_encode([b"x"])
    ch = writer.write_column_chunk(abi.BYTE_ARRAY, [b"abcx"], abi.DELTA_BYTE_ARRAY)
    ch.pages[0].body = data
    res = pqref.decode_batch(writer.build_batch([ch]))
    assert res.status == (abi.ERR_CORRUPT, 0, 0)


def test_dlba_short_data_is_eof():  # in.slice(length) past the end: "Failed to read N bytes"
    ch = writer.write_column_chunk(abi.BYTE_ARRAY, [b"abc", b"defgh"], abi.DELTA_LENGTH_BYTE_ARRAY)
    ch.pages[0].body = ch.pages[0].body[:-2]
    res = pqref.decode_batch(writer.build_batch([ch]))
    assert res.status == (abi.ERR_EOF, 0, 1)


# ---- ByteStreamSplitValuesReaderTest (bytestreamsplit/ByteStreamSplitValuesReaderTest.java) ------------------------

def _bss_page(ptype, body, n, type_length=0):
    ch = writer.write_column_chunk(ptype, np.zeros(n, dtype=abi.numpy_dtype(ptype)) if ptype != abi.FIXED_LEN_BYTE_ARRAY
                                   else [b"\0" * type_length] * n, abi.BYTE_STREAM_SPLIT, type_length=type_length)
    ch.pages[0].body = bytes(body)
    return pqref.decode_batch(writer.build_batch([ch]))


def test_bss_float_small_buffer():  # FloatTest.testSmallBuffer (:64-81)
    body = [0x40, 0x00, 0x80, 0x40, 0x05, 0x84, 0xc5, 0xbd, 0x32, 0xc2, 0x41, 0x42]
    res = _bss_page(abi.FLOAT, body, 3)
    assert res.code == 0
    assert list(res.columns[0]["values"]) == [np.float32(-98.62548828125), np.float32(23.62744140625),
                                              np.float32(44.62939453125)]


def test_bss_double_single_element():  # DoubleTest.testSingleElement
    res = _bss_page(abi.DOUBLE, [0xFE, 0xFF, 0xFF, 0x0D, 0xA8, 0x77, 0xD2, 0x40], 1)
    assert res.code == 0 and float(res.columns[0]["values"][0]) == 18910.62585449218


def test_bss_int_single_element():  # IntegerTest.testSingleElement
    res = _bss_page(abi.INT32, [0x12, 0x34, 0x56, 0x78], 1)
    assert res.code == 0 and int(res.columns[0]["values"][0]) == 0x78563412


def test_bss_float_random_java(  # FloatTest.testRandomInput: java.util.Random(1337).nextFloat() * 1024
):
    r = JavaRandom(1337)
    vals = np.array([r.nextFloat() * np.float32(1024.0) for _ in range(256)], dtype=np.float32)
    res = _decode_bytes(abi.BYTE_STREAM_SPLIT, vals, ptype=abi.FLOAT)
    assert res.code == 0 and np.array_equal(res.columns[0]["values"].view(np.uint32), vals.view(np.uint32))


def test_bss_errors():
    # available % elementSize != 0 -> "Invalid ByteStreamSplit stream" at init (:74-79)
    assert _bss_page(abi.FLOAT, [0] * 7, 2).status == (abi.ERR_CORRUPT, 0, 0)
    # more encoded values than the page's value count (:83-88)
    assert _bss_page(abi.FLOAT, [0] * 12, 2).status == (abi.ERR_CORRUPT, 0, 0)
    # reading past the encoded values: "Byte-stream data was already exhausted." (:43-46)
    assert _bss_page(abi.FLOAT, [0] * 4, 2).status == (abi.ERR_EOF, 0, 1)


# ---- TestBitPacking (parquet-encoding/src/test/.../bitpacking/TestBitPacking.java:36-...): BIG_ENDIAN --------------

BE_CASES = [  # (bit width, values, expected bit string)
    (1, [0], "00000000"), (1, [1], "10000000"), (1, [0, 0], "00000000"), (1, [1, 1], "11000000"),
    (1, [1] * 9, "11111111 10000000"), (1, [0] * 9, "00000000 00000000"),
    (1, [0, 0, 0, 0, 0, 0, 0, 1], "00000001"), (1, [0] * 9 + [1], "00000000 01000000"),
    (1, [0, 1, 0, 0, 1, 1, 1, 0, 0, 1], "01001110 01000000"),
    (2, [0, 1, 2, 3, 3, 3, 2, 1, 1, 0, 0, 0, 1], "00011011 11111001 01000000 01000000"),
]


@pytest.mark.parametrize("w,vals,bits", BE_CASES)
def test_be_bit_packing_known_answers(w, vals, bits):
    expected = bytes(int(b, 2) for b in bits.split())
    assert writer.be_pack(vals, w) == expected
    padded = expected + b"\0" * 16
    got = []
    for g in range(0, len(vals), 8):
        got += list(pqref.unpack8_int_be(w, padded[g * w // 8:]))
    assert got[:len(vals)] == vals


@pytest.mark.parametrize("max_def", [1, 2, 3, 7])
def test_v1_bit_packed_def_levels(max_def):
    """Old parquet-mr V1 pages: BIT_PACKED (big-endian) definition levels, no length prefix."""
    rng = np.random.default_rng(max_def)
    dl = rng.integers(0, max_def + 1, size=5000).astype(np.uint8)
    vals = np.arange(int((dl == max_def).sum()), dtype=np.int64)
    ch = writer.write_column_chunk(abi.INT64, vals, abi.PLAIN, def_levels=dl, max_def=max_def, version=1,
                                   level_encoding=abi.BIT_PACKED, page_rows=1000)
    res = pqref.decode_batch(writer.build_batch([ch]))
    assert res.code == 0, res.status
    assert np.array_equal(res.columns[0]["def_levels"], dl) and np.array_equal(res.columns[0]["values"], vals)
