"""PARQUET-246 carry-over (PQG_PAGE_DBA_CARRY) and DELTA_BYTE_ARRAY on FIXED_LEN_BYTE_ARRAY.

Follows parquet-column's TestCorruptDeltaByteArrays
(src/test/java/org/apache/parquet/column/impl/TestCorruptDeltaByteArrays.java): the created_by
classification (testCorruptDeltaByteArrayVerisons, testEncodingRequiresSequentailRead), a page written
with the previous page's last value still in the writer (corruptWriter, str(i) = "aaaaaaaaaaa" + char)
read without the carry-over (AIOOBE -> PQG_ERR_CORRUPT) and with it (testReassemblyWithCorruptPage,
testColumnReaderImplWithCorruptPage), and uncorrupted pages read with and without it
(testReassemblyWithoutCorruption, testOldReassemblyWithoutCorruption). The oracle (CPU, test
infrastructure) is checked here; the `gpu` tests compare the device path with it bit for bit."""
import numpy as np
import pytest

from oracle import pqref
from pqgpu import abi
from tools.synth import writer
from pqgpu.version import requires_sequential_reads

from helpers import assert_same


def jstr(i):
    return b"aaaaaaaaaaa" + bytes([ord("a") + i])


# ---- created_by -> carry-over (CorruptDeltaByteArrays) --------------------------------------------------

@pytest.mark.parametrize("created_by,encoding,expect", [
    ("parquet-mr version 1.6.0 (build abcd)", abi.DELTA_BYTE_ARRAY, True),
    (None, abi.DELTA_BYTE_ARRAY, True),
    ("", abi.DELTA_BYTE_ARRAY, True),
    ("parquet-mr version 1.8.0-SNAPSHOT (build abcd)", abi.DELTA_BYTE_ARRAY, True),
    ("parquet-mr version 1.6.0 (build abcd)", abi.DELTA_BINARY_PACKED, False),
    (None, abi.DELTA_LENGTH_BYTE_ARRAY, False),
    (None, abi.PLAIN, False),
    (None, abi.RLE, False),
    ("parquet-mr version 1.8.0-SNAPSHOT (build abcd)", abi.RLE_DICTIONARY, False),
    ("parquet-mr version 1.8.0-SNAPSHOT (build abcd)", abi.PLAIN_DICTIONARY, False),
    ("parquet-mr version 1.8.0-SNAPSHOT (build abcd)", abi.BIT_PACKED, False),
    ("parquet-mr version 1.8.0 (build abcd)", abi.DELTA_BYTE_ARRAY, False),
    # testEncodingRequiresSequentailRead: ParsedVersion(app, version, build)
    ("impala version 1.2.0 (build abcd)", abi.DELTA_BYTE_ARRAY, False),
    ("parquet-mr version 1.8.0rc2-SNAPSHOT (build ddb4)", abi.DELTA_BYTE_ARRAY, True),  # VersionParser example
    ("parquet-mr version 1.8.0rc2", abi.DELTA_BYTE_ARRAY, True),         # unknown part sorts before 1.8.0
    ("parquet-mr version 1.7.9 (build x)", abi.DELTA_BYTE_ARRAY, True),
    ("parquet-mr version 1.10.1 (build x)", abi.DELTA_BYTE_ARRAY, False),
    ("parquet-mr version 1.13.1 (build db4183109d5b734ec5930d870cdae161e408ddba)", abi.DELTA_BYTE_ARRAY, False),
    ("parquet-mr version not-a-version", abi.DELTA_BYTE_ARRAY, True),   # no semantic version
    ("parquet-mr", abi.DELTA_BYTE_ARRAY, True),                          # does not parse
    ("parquet-cpp-arrow version 14.0.1", abi.DELTA_BYTE_ARRAY, False),
])
def test_requires_sequential_reads(created_by, encoding, expect):
    assert requires_sequential_reads(created_by, encoding) is expect


# ---- oracle ---------------------------------------------------------------------------------------------

def two_pages(corrupt, flag):
    """Ten values str(0..9), then str(10..19) written with `previous` = str(9) when corrupt."""
    vals = [jstr(i) for i in range(20)]
    ch = writer.write_column_chunk(abi.BYTE_ARRAY, vals, abi.DELTA_BYTE_ARRAY, page_rows=10, dba_carry=corrupt)
    ch.dba_carry = flag
    return vals, writer.build_batch([ch])


def test_written_pages_match_the_reference_writer():
    """The corrupt page's first value shares 11 bytes with str(9); an uncorrupted one shares none."""
    vals, b = two_pages(True, True)
    assert list(b.pages["flags"]) == [0, abi.PAGE_DBA_CARRY]
    body = b.data[int(b.pages["offset"][1]): int(b.pages["offset"][1]) + int(b.pages["size"][1])].tobytes()
    assert pqref.delta_decode(body)[0][0] == 11
    _, b2 = two_pages(False, False)
    body2 = b2.data[int(b2.pages["offset"][1]): int(b2.pages["offset"][1]) + int(b2.pages["size"][1])].tobytes()
    assert pqref.delta_decode(body2)[0][0] == 0


def test_oracle_corrupt_page_without_carry_fails():
    _, b = two_pages(True, False)
    r = pqref.decode_batch(b)
    assert r.status == (abi.ERR_CORRUPT, 1, 0)


@pytest.mark.parametrize("corrupt", [True, False])
def test_oracle_carry(corrupt):
    vals, b = two_pages(corrupt, True)
    r = pqref.decode_batch(b)
    assert r.code == 0, r.status
    assert r.columns[0]["values"] == vals


def test_oracle_carry_after_a_non_dba_page_is_unsupported():
    """setPreviousReader casts the previous page's reader to DeltaByteArrayReader."""
    vals = [jstr(i % 20) for i in range(40)]
    a = writer.write_column_chunk(abi.BYTE_ARRAY, vals[:20], abi.PLAIN, page_rows=20)
    c = writer.write_column_chunk(abi.BYTE_ARRAY, vals[20:], abi.DELTA_BYTE_ARRAY, page_rows=20)
    a.pages += c.pages
    a.values = vals
    b = writer.build_batch([a])
    b.pages["flags"][1] = abi.PAGE_DBA_CARRY
    assert pqref.decode_batch(b).status == (abi.ERR_UNSUPPORTED, 1, 0)


def carry_column(n, page_rows, seed, nullable=False, long_every=0, physical_type=abi.BYTE_ARRAY, width=0):
    rng = np.random.default_rng(seed)
    keys = np.sort(rng.integers(0, 10**9, size=n))
    vals = [b"https://example.org/item/" + b"%012d" % k for k in keys]
    if long_every:
        vals = [v + b"L" * 3000 if i % long_every == long_every - 1 else v for i, v in enumerate(vals)]
    if physical_type == abi.FIXED_LEN_BYTE_ARRAY:
        vals = [v[-width:] for v in vals]
    dl = None
    if nullable:
        dl = (rng.random(n) > 0.3).astype(np.uint8)
        dl[page_rows:2 * page_rows] = 0  # one null-only page
        vals = [v for v, d in zip(vals, dl) if d]
    return writer.write_column_chunk(physical_type, vals, abi.DELTA_BYTE_ARRAY, page_rows=page_rows,
                                     def_levels=dl, max_def=1 if nullable else 0, dba_carry=True,
                                     type_length=width), vals


@pytest.mark.parametrize("nullable", [False, True])
def test_oracle_carry_many_pages(nullable):
    ch, vals = carry_column(5000, 300, 1, nullable=nullable)
    r = pqref.decode_batch(writer.build_batch([ch]))
    assert r.code == 0 and r.columns[0]["values"] == vals
    ch.dba_carry = False  # the same pages without the carry-over fail at the first carried prefix
    r = pqref.decode_batch(writer.build_batch([ch]))
    assert r.code == abi.ERR_CORRUPT


def test_oracle_flba_dba():
    ch, vals = carry_column(3000, 700, 2, physical_type=abi.FIXED_LEN_BYTE_ARRAY, width=9)
    ch.dba_carry = False
    ch2 = writer.write_column_chunk(abi.FIXED_LEN_BYTE_ARRAY, vals, abi.DELTA_BYTE_ARRAY, page_rows=700, type_length=9)
    r = pqref.decode_batch(writer.build_batch([ch2]))
    assert r.code == 0
    assert [bytes(v) for v in r.columns[0]["values"]] == vals
    bad = writer.write_column_chunk(abi.FIXED_LEN_BYTE_ARRAY, vals[:100] + [b"short"] + vals[101:200],
                                    abi.DELTA_BYTE_ARRAY, page_rows=64, type_length=9)
    assert pqref.decode_batch(writer.build_batch([bad])).status == (abi.ERR_CORRUPT, 1, 36)


# ---- device vs oracle ------------------------------------------------------------------------------------

def run_both(decoder, batch, expect_code=0):
    ref = pqref.decode_batch(batch)
    dcols, st = decoder.decode(decoder.upload(batch), check=False)
    assert (int(st.code), int(st.page), int(st.value_index)) == ref.status, (st.message, ref.status)
    assert ref.code == expect_code, ref.status
    if expect_code:
        return
    for i, cd in enumerate(batch.columns):
        assert dcols[i].n_values == ref.columns[i]["n_values"]
        assert_same(dcols[i].numpy(), ref.columns[i]["values"], cd["physical_type"])
        if cd["max_def"] > 0:
            assert np.array_equal(dcols[i].def_levels[:batch.column_slots[i]].cpu().numpy(), ref.columns[i]["def_levels"])


@pytest.mark.gpu
@pytest.mark.parametrize("corrupt,flag,code", [(True, True, 0), (True, False, abi.ERR_CORRUPT), (False, True, 0),
                                               (False, False, 0)])
def test_gpu_reference_cases(decoder, corrupt, flag, code):
    _, b = two_pages(corrupt, flag)
    run_both(decoder, b, code)


@pytest.mark.gpu
@pytest.mark.parametrize("nullable", [False, True])
@pytest.mark.parametrize("long_every", [0, 97])
def test_gpu_carry_many_pages(decoder, nullable, long_every):
    """300-value pages carried one into the next (a null-only page in the nullable case, values over
    the 2 KiB LDS value buffer when long_every), next to an unflagged copy of the same column and
    two row groups of one output column (the carry restarts at the second chunk's first page)."""
    ch, vals = carry_column(6000, 300, 3, nullable=nullable, long_every=long_every)
    plain, _ = carry_column(6000, 300, 3, nullable=nullable, long_every=long_every)
    plain.dba_carry = False  # decoded on the chunk-parallel path; its carried prefixes fail
    g1, _ = carry_column(2000, 250, 5)
    g2, _ = carry_column(2000, 250, 6)
    g1.column_index = g2.column_index = "rg"
    run_both(decoder, writer.build_batch([ch, g1, g2]))
    run_both(decoder, writer.build_batch([ch, plain]), abi.ERR_CORRUPT)


@pytest.mark.gpu
def test_gpu_carry_after_non_dba_page(decoder):
    vals = [jstr(i % 20) for i in range(40)]
    a = writer.write_column_chunk(abi.BYTE_ARRAY, vals[:20], abi.PLAIN, page_rows=20)
    c = writer.write_column_chunk(abi.BYTE_ARRAY, vals[20:], abi.DELTA_BYTE_ARRAY, page_rows=20)
    a.pages += c.pages
    a.values = vals
    b = writer.build_batch([a])
    b.pages["flags"][1] = abi.PAGE_DBA_CARRY
    run_both(decoder, b, abi.ERR_UNSUPPORTED)


@pytest.mark.gpu
@pytest.mark.parametrize("width", [1, 9, 16, 33])
def test_gpu_flba_dba(decoder, width):
    ch, vals = carry_column(20000, 3000, 7, physical_type=abi.FIXED_LEN_BYTE_ARRAY, width=width)
    ch2 = writer.write_column_chunk(abi.FIXED_LEN_BYTE_ARRAY, vals, abi.DELTA_BYTE_ARRAY, page_rows=3000,
                                    type_length=width)
    run_both(decoder, writer.build_batch([ch2]))
    run_both(decoder, writer.build_batch([ch]))  # PARQUET-246 pages on FLBA


@pytest.mark.gpu
def test_gpu_flba_dba_wrong_length(decoder):
    _, vals = carry_column(3000, 700, 2, physical_type=abi.FIXED_LEN_BYTE_ARRAY, width=9)
    bad = writer.write_column_chunk(abi.FIXED_LEN_BYTE_ARRAY, vals[:100] + [b"short"] + vals[101:2000],
                                    abi.DELTA_BYTE_ARRAY, page_rows=64, type_length=9)
    run_both(decoder, writer.build_batch([bad]), abi.ERR_CORRUPT)
