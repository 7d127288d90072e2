"""GPU parity: libpqgpu.so (through the C ABI) vs the oracle on the same pages.

Bit-exact on values (floats compared as bit patterns), levels, per-page value
counts and the first error (code, page, index). Cases follow the reference's
tests and BASELINE.json's configs at oracle-friendly sizes.
"""
import numpy as np
import pytest

from oracle import pqref
from pqgpu import abi
from tools.synth import writer

from helpers import assert_same, make, nulls, zipf_dict_column

pytestmark = pytest.mark.gpu


def run_both(decoder, chunks, expect_error=False):
    batch = writer.build_batch(chunks)
    ref = pqref.decode_batch(batch)
    dcols, st = decoder.decode(decoder.upload(batch), check=False)
    assert (int(st.code), int(st.page), int(st.value_index)) == ref.status, \
        f"gpu status {st.code, st.page, st.value_index} {st.message} vs oracle {ref.status}"
    if expect_error:
        assert ref.code != 0
        return batch, ref, dcols
    assert ref.code == 0, ref.status
    for i, cd in enumerate(batch.columns):
        col = dcols[i]
        assert col.n_values == ref.columns[i]["n_values"]
        assert_same(col.numpy(), ref.columns[i]["values"], cd["physical_type"])
        if cd["physical_type"] == abi.BYTE_ARRAY:
            assert np.array_equal(col.offsets().cpu().numpy(), ref.columns[i]["offsets"][:col.n_values + 1])
        if cd["max_def"] > 0:
            assert np.array_equal(col.def_levels[:batch.column_slots[i]].cpu().numpy(), ref.columns[i]["def_levels"])
        if cd["max_rep"] > 0:
            assert np.array_equal(col.rep_levels[:batch.column_slots[i]].cpu().numpy(), ref.columns[i]["rep_levels"])
    return batch, ref, dcols


# ---- config 2 shape: RLE_DICTIONARY int64, Zipf run lengths --------------------------------------------

@pytest.mark.parametrize("a", [1.5, 2.0, 3.0])
@pytest.mark.parametrize("card", [1, 2, 1000, 70000])
def test_dict_int64_zipf(decoder, a, card):
    vals = zipf_dict_column(200_000, card=card, a=a, seed=int(a * 10) + card)
    run_both(decoder, [make(abi.INT64, vals, abi.RLE_DICTIONARY)])


@pytest.mark.parametrize("ptype", [abi.INT32, abi.FLOAT, abi.DOUBLE])
def test_dict_other_types(decoder, ptype):
    vals = zipf_dict_column(120_000, card=300, a=1.7, seed=3, physical_type=ptype)
    run_both(decoder, [make(ptype, vals, abi.PLAIN_DICTIONARY, dict_page_encoding=abi.PLAIN_DICTIONARY)])


@pytest.mark.parametrize("page_rows", [1, 7, 8, 9, 504, 505, 20000])
def test_dict_page_sizes(decoder, page_rows):
    vals = zipf_dict_column(30_000, card=50, a=1.3, seed=page_rows)
    run_both(decoder, [make(abi.INT64, vals, abi.RLE_DICTIONARY, page_rows=page_rows)])


def test_dict_multiple_columns_interleaved(decoder):
    chunks = []
    for k in range(4):
        v = zipf_dict_column(50_000, card=10 + k * 200, a=1.5 + 0.2 * k, seed=k,
                             physical_type=abi.INT64 if k % 2 == 0 else abi.INT32)
        chunks.append(make(abi.INT64 if k % 2 == 0 else abi.INT32, v, abi.RLE_DICTIONARY, page_rows=7000))
    batch = writer.build_batch(chunks)
    # interleave pages of the 4 columns (page order within a column kept)
    order = np.argsort(np.arange(batch.n_pages) % 7, kind="stable")
    cols = batch.pages["column"][order]
    for c in range(4):  # keep per-column order
        idx = np.nonzero(cols == c)[0]
        order[idx] = np.sort(order[idx])
    batch.pages = batch.pages[order]
    batch.page_slot_offsets = batch.page_slot_offsets[order]
    ref = pqref.decode_batch(batch)
    dcols, st = decoder.decode(decoder.upload(batch), check=False)
    assert st.code == 0 and ref.code == 0
    for i in range(4):
        assert_same(dcols[i].numpy(), ref.columns[i]["values"], batch.columns[i]["physical_type"])


@pytest.mark.parametrize("case", ["multi", "many_pages", "id_error", "tiny"])
def test_dict_columns_of_both_widths(decoder, case):
    """Several fused dictionary columns of both widths in one launch, a column of fewer chunks than an
    expansion workgroup, and a dictionary-id error beside a truncated page: values and first error as the
    oracle's."""
    if case == "tiny":
        chunks = [make(abi.INT32, zipf_dict_column(37, card=5, a=1.5, seed=1, physical_type=abi.INT32),
                       abi.RLE_DICTIONARY, page_rows=10)]
    elif case == "many_pages":
        chunks = [make(abi.INT64, zipf_dict_column(300_000, card=900, a=1.2, seed=2), abi.RLE_DICTIONARY,
                       page_rows=1500)]
    else:
        chunks = []
        for k in range(5):
            pt = abi.INT64 if k % 2 == 0 else abi.INT32
            v = zipf_dict_column(40_000 + 9_000 * k, card=3 + k * 300, a=1.4 + 0.3 * k, seed=10 + k, physical_type=pt)
            chunks.append(make(pt, v, abi.RLE_DICTIONARY, page_rows=3000 + 1000 * k))
    if case == "id_error":
        chunks[3].dict_num_values = 600  # ids >= 600 of column 3 out of range; truncated page in column 1
        chunks[1].pages[5].body = chunks[1].pages[5].body[:-7]
        run_both(decoder, chunks, expect_error=True)
    else:
        run_both(decoder, chunks)


def test_dict_known_answer_pages(decoder):
    """TestDictionary.testLongDictionary (:285-317): 1000 x (i % 50), then 2000 descending."""
    v1 = np.arange(1000, dtype=np.int64) % 50
    v2 = np.arange(2000, 0, -1, dtype=np.int64) % 50
    ch = make(abi.INT64, np.concatenate([v1, v2]), abi.PLAIN_DICTIONARY, page_rows=1000)
    batch, ref, dcols = run_both(decoder, [ch])
    assert np.array_equal(dcols[0].numpy(), np.concatenate([v1, v2]))


# ---- nulls / levels (configs 3 and 5) -------------------------------------------------------------------

@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("enc,ptype", [(abi.RLE_DICTIONARY, abi.INT64), (abi.PLAIN, abi.DOUBLE),
                                       (abi.PLAIN, abi.INT32), (abi.DELTA_BINARY_PACKED, abi.INT64),
                                       (abi.DELTA_BINARY_PACKED, abi.INT32), (abi.PLAIN, abi.BOOLEAN)])
@pytest.mark.parametrize("null_frac", [0.0, 0.1, 0.9, 1.0])
def test_optional_columns(decoder, version, enc, ptype, null_frac):
    n_slots = 50_000
    dl = nulls(n_slots, null_frac, seed=5)
    n = int(dl.sum())
    rng = np.random.default_rng(11)
    if enc == abi.RLE_DICTIONARY:
        vals = zipf_dict_column(max(n, 1), card=500, seed=2)[:n]
    elif ptype == abi.DOUBLE:
        vals = rng.standard_normal(n)
    elif ptype == abi.BOOLEAN:
        vals = rng.integers(0, 2, size=n).astype(np.uint8)
    elif enc == abi.DELTA_BINARY_PACKED and ptype == abi.INT64:
        vals = np.cumsum(rng.integers(-1000, 100000, size=n)).astype(np.int64)
    else:
        vals = rng.integers(-2**31, 2**31 - 1, size=n).astype(np.int32)
    ch = make(ptype, vals, enc, def_levels=dl, max_def=1, version=version, page_rows=20000)
    run_both(decoder, [ch])


@pytest.mark.parametrize("version", [1, 2])
def test_nested_list_levels(decoder, version):
    """Config 5 shape: optional group (LIST) { repeated group list { optional int64 element } }:
    max_rep 1, max_def 3. Lists ~ Poisson(3), 10% null lists, 10% null elements."""
    rng = np.random.default_rng(11)
    recs = 20_000
    lens = rng.poisson(3, size=recs)
    null_list = rng.random(recs) < 0.1
    rl, dl = [], []
    for L, nl in zip(lens, null_list):
        if nl:
            rl.append(0); dl.append(0)
        elif L == 0:
            rl.append(0); dl.append(1)
        else:
            for j in range(L):
                rl.append(0 if j == 0 else 1)
                dl.append(3 if rng.random() >= 0.1 else 2)
    rl = np.array(rl, dtype=np.uint8)
    dl = np.array(dl, dtype=np.uint8)
    n = int((dl == 3).sum())
    vals = rng.integers(-2**40, 2**40, size=n).astype(np.int64)
    ch = make(abi.INT64, vals, abi.PLAIN, def_levels=dl, rep_levels=rl, max_def=3, max_rep=1, version=version,
              page_rows=5000)
    run_both(decoder, [ch])


# ---- PLAIN (config 1 shape) and DELTA (config 3 shape) ----------------------------------------------------

@pytest.mark.parametrize("ptype", [abi.INT32, abi.INT64, abi.FLOAT, abi.DOUBLE, abi.BOOLEAN])
@pytest.mark.parametrize("n", [0, 1, 15, 1_000_000])
def test_plain_required(decoder, ptype, n):
    rng = np.random.default_rng(n)
    dt = abi.numpy_dtype(ptype)
    if ptype == abi.BOOLEAN:
        vals = rng.integers(0, 2, size=n).astype(np.uint8)
    else:
        vals = rng.integers(0, 255, size=n * dt.itemsize, dtype=np.uint8).view(dt)
    run_both(decoder, [make(ptype, vals, abi.PLAIN, page_rows=20000)])


@pytest.mark.parametrize("ptype,w", [(abi.FIXED_LEN_BYTE_ARRAY, 3), (abi.FIXED_LEN_BYTE_ARRAY, 16),
                                     (abi.INT96, 12)])
def test_plain_fixed_len(decoder, ptype, w):
    rng = np.random.default_rng(w)
    vals = [rng.integers(0, 255, size=w, dtype=np.uint8).tobytes() for _ in range(5000)]
    run_both(decoder, [make(ptype, vals, abi.PLAIN, type_length=w if ptype == abi.FIXED_LEN_BYTE_ARRAY else 0,
                            page_rows=999)])


@pytest.mark.parametrize("ptype", [abi.INT32, abi.INT64])
@pytest.mark.parametrize("kind", ["walk", "random", "minmax", "const", "short"])
def test_delta(decoder, ptype, kind):
    rng = np.random.default_rng(7)
    n = 100_003
    info = np.iinfo(np.int64 if ptype == abi.INT64 else np.int32)
    if kind == "walk":
        vals = np.cumsum(rng.integers(-50, 500, size=n))
    elif kind == "random":
        vals = rng.integers(info.min, info.max, size=n, dtype=np.int64)
    elif kind == "minmax":  # DeltaBinaryPackingValuesWriterForLongTest.shouldReadMaxMinValue (:130-141)
        vals = np.where(np.arange(n) % 2 == 0, info.min, info.max)
    elif kind == "const":
        vals = np.full(n, 3)
    else:
        n = 29
        vals = rng.integers(-10, 10, size=n)
    vals = vals.astype(np.int64 if ptype == abi.INT64 else np.int32)
    run_both(decoder, [make(ptype, vals, abi.DELTA_BINARY_PACKED, page_rows=20000)])


@pytest.mark.parametrize("ptype", [abi.INT32, abi.INT64])
@pytest.mark.parametrize("page_rows", [20001, 20003, 513, 1023])
def test_delta_output_shifts(decoder, ptype, page_rows):
    # pages of an odd value count start at every output offset mod 16 bytes, so the expansion's
    # transposed 1 KiB rows run at every shift (4-byte values: 0..3, the last row of a step cut at
    # lane 63's last value for shifts 2 and 3) and pages of ~1 / ~2 full 512-value steps end in partial ones
    rng = np.random.default_rng(page_rows)
    n = 8 * page_rows + 77
    vals = np.cumsum(rng.integers(-50, 1 << 12, size=n)).astype(np.int64 if ptype == abi.INT64 else np.int32)
    run_both(decoder, [make(ptype, vals, abi.DELTA_BINARY_PACKED, page_rows=page_rows)])


@pytest.mark.parametrize("ptype", [abi.INT32, abi.INT64])
@pytest.mark.parametrize("block,mb", [(2048, 8), (1024, 4), (768, 3)])
@pytest.mark.parametrize("kind", ["walk", "random", "mixed"])
def test_delta_big_blocks(decoder, ptype, block, mb, kind):
    # blocks of 513..2048 values take the batched walk and segment expansion while a block's deltas fit the
    # LDS segment (8 KiB); 64-bit random deltas (16 KiB per 2048-value block) fall back to the block-by-block
    # path from that block on ("mixed": small deltas first, random ones after, so one page takes both)
    rng = np.random.default_rng(block + mb)
    n = 45_001
    info = np.iinfo(np.int64 if ptype == abi.INT64 else np.int32)
    if kind == "walk":
        vals = np.cumsum(rng.integers(-50, 5000, size=n))
    elif kind == "random":
        vals = rng.integers(info.min, info.max, size=n, dtype=np.int64)
    else:
        vals = np.concatenate([np.cumsum(rng.integers(-50, 5000, size=n // 2)),
                               rng.integers(info.min, info.max, size=n - n // 2, dtype=np.int64)])
    vals = vals.astype(np.int64 if ptype == abi.INT64 else np.int32)
    run_both(decoder, [make(ptype, vals, abi.DELTA_BINARY_PACKED, delta_block=block, delta_miniblocks=mb,
                            page_rows=15_000)])


@pytest.mark.parametrize("block,mb", [(128, 4), (64, 8), (256, 8), (512, 8), (32, 1), (8, 1),
                                      (192, 3), (24, 3), (320, 5),
                                      # block-by-block path: > 512 values or > 8 miniblocks (DuckDB: 2048 / 8)
                                      (1024, 4), (2048, 8), (128, 16), (1024, 128), (40000, 5), (8192, 64)])
@pytest.mark.parametrize("ptype", [abi.INT64, abi.INT32])
def test_delta_configs(decoder, block, mb, ptype):
    # blocks of 8 * 2^k values take the several-blocks-per-step expansion, the others one block per
    # step; blocks of more than 512 values or more than 8 miniblocks the block-by-block path
    rng = np.random.default_rng(block)
    vals = np.cumsum(rng.integers(-3, 1 << 20, size=40_000)).astype(np.int64)
    if ptype == abi.INT32:
        vals = vals.astype(np.int32)
    run_both(decoder, [make(ptype, vals, abi.DELTA_BINARY_PACKED, delta_block=block, delta_miniblocks=mb)])


# ---- error classification ----------------------------------------------------------------------------

def _dict_chunk(n=5000, card=100, seed=1):
    return make(abi.INT64, zipf_dict_column(n, card=card, a=1.5, seed=seed), abi.RLE_DICTIONARY, page_rows=1000)


def test_error_dict_id_out_of_range(decoder):
    ch = _dict_chunk()
    ch.dict_num_values = 10  # ids >= 10 now out of range (AIOOBE in decodeToLong)
    run_both(decoder, [ch], expect_error=True)


def test_error_bit_width(decoder):
    ch = _dict_chunk()
    pg = ch.pages[2]
    pg.body = bytes([33]) + pg.body[1:]
    run_both(decoder, [ch], expect_error=True)


@pytest.mark.parametrize("cut", [1, 2, 5, 40])
def test_error_truncated_page(decoder, cut):
    ch = _dict_chunk(card=1000, seed=4)
    pg = ch.pages[3]
    pg.body = pg.body[:max(1, len(pg.body) - cut)]
    batch, ref, _ = run_both(decoder, [ch], expect_error=ref_errors(ch))


def ref_errors(ch):
    return pqref.decode_batch(writer.build_batch([ch])).code != 0


def test_error_empty_page(decoder):
    ch = _dict_chunk()
    ch.pages[1].body = b""
    run_both(decoder, [ch], expect_error=True)


def test_error_plain_eof(decoder):
    ch = make(abi.INT64, np.arange(5000, dtype=np.int64), abi.PLAIN, page_rows=1000)
    ch.pages[2].body = ch.pages[2].body[:-12]
    run_both(decoder, [ch], expect_error=True)


def test_error_delta_past_end(decoder):
    ch = make(abi.INT64, np.arange(3000, dtype=np.int64), abi.DELTA_BINARY_PACKED, page_rows=1000)
    ch.pages[1].num_values = 1500  # header total is 1000
    run_both(decoder, [ch], expect_error=True)


@pytest.mark.parametrize("block,mb", [(128, 4), (2048, 8), (256, 32)])
@pytest.mark.parametrize("cut", [1, 3, 17, 300, 1500])
def test_error_delta_truncated(decoder, block, mb, cut):
    # truncated DELTA pages: the batched and the block-by-block paths classify like the oracle
    vals = np.cumsum(np.random.default_rng(cut).integers(-3, 1 << 30, size=6000)).astype(np.int64)
    ch = make(abi.INT64, vals, abi.DELTA_BINARY_PACKED, page_rows=3000, delta_block=block, delta_miniblocks=mb)
    ch.pages[1].body = ch.pages[1].body[:len(ch.pages[1].body) - cut]
    run_both(decoder, [ch], expect_error=ref_errors(ch))


def test_error_delta_wide_miniblock(decoder):
    # a miniblock width over 64 (CORRUPT) in a block of the block-by-block path
    ch = make(abi.INT64, np.arange(5000, dtype=np.int64) * 7, abi.DELTA_BINARY_PACKED, page_rows=5000,
              delta_block=1024, delta_miniblocks=8)
    body = bytearray(ch.pages[0].body)
    # header varints: block, miniblocks, total, first (zigzag 0 = 1 byte); then block 0: min delta (1 byte), widths
    hdr = 2 + 1 + 2 + 1
    body[hdr + 1 + 2] = 65
    ch.pages[0].body = bytes(body)
    run_both(decoder, [ch], expect_error=True)


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("kind", ["runs", "random", "nulls"])
def test_rle_boolean(decoder, version, kind):
    # BOOLEAN values with encoding RLE (parquet-mr's V2 writer for booleans)
    rng = np.random.default_rng(len(kind) * 10 + version)
    n = 50_000
    if kind == "runs":
        vals = np.repeat(rng.random(2000) < 0.5, np.minimum(rng.zipf(1.3, size=2000), 5000))[:n]
    else:
        vals = rng.random(n) < 0.4
    dl = nulls(len(vals), 0.25, seed=3) if kind == "nulls" else None
    v = vals[dl.astype(bool)] if dl is not None else vals
    ch = make(abi.BOOLEAN, v.astype(np.uint8), abi.RLE, def_levels=dl, max_def=1 if dl is not None else 0,
              version=version, page_rows=7000)
    run_both(decoder, [ch])


def test_rle_boolean_unmasked_run_value(decoder):
    # an RLE run's repeated byte is not masked to the width: readBoolean = (value != 0)
    rle = bytes([20 << 1, 0x02, 10 << 1, 0x00, 5 << 1, 0xFF, 1 << 1 | 1, 0b10110010])  # 20 x 2, 10 x 0, 5 x 255, 8 bits
    ch = make(abi.BOOLEAN, np.zeros(43, dtype=np.uint8), abi.RLE)
    ch.pages[0].body = len(rle).to_bytes(4, "little") + rle
    _, ref, _ = run_both(decoder, [ch])
    assert list(ref.columns[0]["values"]) == [1] * 20 + [0] * 10 + [1] * 5 + [0, 1, 0, 0, 1, 1, 0, 1]


@pytest.mark.parametrize("cut", [1, 2, 4, 9, 60])
def test_error_rle_boolean_truncated(decoder, cut):
    vals = (np.random.default_rng(cut).random(9000) < 0.5).astype(np.uint8)
    ch = make(abi.BOOLEAN, vals, abi.RLE, page_rows=3000)
    ch.pages[1].body = ch.pages[1].body[:max(0, len(ch.pages[1].body) - cut)]
    run_both(decoder, [ch], expect_error=ref_errors(ch))


def test_error_rle_boolean_length(decoder):
    vals = (np.arange(3000) % 3 == 0).astype(np.uint8)
    for bad in (-5, 10**6, 2):  # negative length, past the page, shorter than the values need
        ch = make(abi.BOOLEAN, vals, abi.RLE, page_rows=1000)
        body = bytearray(ch.pages[1].body)
        body[0:4] = int(bad).to_bytes(4, "little", signed=True)
        ch.pages[1].body = bytes(body)
        run_both(decoder, [ch], expect_error=True)


def test_error_missing_dictionary(decoder):
    ch = _dict_chunk()
    ch.dict_page = None
    run_both(decoder, [ch], expect_error=True)


@pytest.mark.parametrize("seed", range(16))
def test_error_level_sections_corrupted(decoder, seed):
    """Level sections with bytes overwritten at random, or cut short (V2: the section lengths of the
    header kept, V1: the length prefix kept): the first error (code, page, slot) or, with none, the
    levels and values equal the oracle's. Nested (rep + def) columns for seeds 2, 3 mod 4."""
    rng = np.random.default_rng(seed)
    version = 1 + seed % 2
    n = 8000
    if seed % 4 < 2:
        dl = nulls(n, 0.3, seed=seed)
        rl, max_def, max_rep = None, 1, 0
    else:
        rl = (rng.random(n) < 0.6).astype(np.uint8)
        rl[0] = 0
        dl = rng.integers(0, 4, size=n).astype(np.uint8)
        max_def, max_rep = 3, 1
    vals = rng.integers(-2**31, 2**31 - 1, size=int((dl == max_def).sum())).astype(np.int32)
    ch = make(abi.INT32, vals, abi.PLAIN, def_levels=dl, rep_levels=rl, max_def=max_def, max_rep=max_rep,
              version=version, page_rows=1000)
    for pg in ch.pages:
        body = bytearray(pg.body)
        if version == 2:
            lo, hi = 0, pg.rl_byte_length + pg.dl_byte_length
        else:
            lo, hi = 4, min(len(body), 4 + int.from_bytes(body[0:4], "little"))
        if hi <= lo:
            continue
        k = rng.integers(0, 4)
        for _ in range(k):
            body[rng.integers(lo, hi)] = int(rng.integers(0, 256))
        if rng.random() < 0.2 and version == 2:  # its last bytes zeroed
            cut = int(rng.integers(1, max(2, (hi - lo) // 2)))
            body[hi - cut:hi] = bytes(cut)
        pg.body = bytes(body)
    batch = writer.build_batch([ch])
    ref = pqref.decode_batch(batch)
    run_both(decoder, [ch], expect_error=ref.code != 0)


def test_error_level_section_length(decoder):
    dl = nulls(4000, 0.2, seed=1)
    ch = make(abi.DOUBLE, np.random.default_rng(0).standard_normal(int(dl.sum())), abi.PLAIN, def_levels=dl,
              max_def=1, version=1, page_rows=1000)
    body = bytearray(ch.pages[1].body)
    body[0:4] = (len(body) + 10).to_bytes(4, "little")
    ch.pages[1].body = bytes(body)
    run_both(decoder, [ch], expect_error=True)


# ---- ParquetReadRouter -------------------------------------------------------------------------------

@pytest.mark.parametrize("w", list(range(0, 33)))
def test_router_read(decoder, w):
    rng = np.random.default_rng(w)
    count = 2048
    data = rng.integers(0, 256, size=count * w // 8 + 3, dtype=np.uint8)
    got = decoder.router_read(w, data, count)
    ref, _ = pqref.router_read(w, data, count)
    assert np.array_equal(got, ref)


def test_host_path_roundtrip(decoder):
    vals = zipf_dict_column(100_000, card=1000, seed=9)
    batch = writer.build_batch([make(abi.INT64, vals, abi.RLE_DICTIONARY)])
    rc, st, res, counts = decoder.decode_host(batch)
    assert rc == 0, st.message
    assert np.array_equal(res[0]["values"], vals)
    assert counts.sum() == vals.size


@pytest.mark.parametrize("what", ["page", "dictionary"])
@pytest.mark.parametrize("over", [1, 100, 1023])
def test_host_path_extent_past_buffer(decoder, what, over):
    """pqg_decode_host reads its staged bytes with 1 KiB of zero padding; a page or dictionary whose
    extent runs past the CALLER's buffer by fewer than 1 KiB must still be rejected (INVALID_ARG),
    as pqg_decode rejects it, not decoded against the padding (the reference would hit EOF)."""
    import copy
    vals = zipf_dict_column(40_000, card=300, seed=11)
    batch = writer.build_batch([make(abi.INT64, vals, abi.RLE_DICTIONARY)])
    b = copy.copy(batch)
    b.pages = batch.pages.copy()
    b.columns = [dict(c) for c in batch.columns]
    n = batch.data.size
    if what == "page":
        p = b.n_pages - 1
        b.pages["size"][p] = n - int(b.pages["offset"][p]) + over
    else:
        b.columns[0]["dict_size"] = n - int(b.columns[0]["dict_offset"]) + over
    rc, st, res, counts = decoder.decode_host(b)
    assert rc == abi.ERR_INVALID_ARG, (rc, st.message)
    if what == "page":
        assert st.page == b.n_pages - 1
    rc, st, res, counts = decoder.decode_host(batch)
    assert rc == 0 and np.array_equal(res[0]["values"], vals)


@pytest.mark.parametrize("max_def", [1, 2, 5, 12, 20, 40])
@pytest.mark.parametrize("shape", ["random", "runs"])
@pytest.mark.parametrize("version", [1, 2])
def test_rle_level_widths(decoder, max_def, shape, version):
    """RLE / bit-packed hybrid definition levels of bit widths 1..6 (the level expansion is
    specialised per width up to 4), random (mostly bit-packed) and run-heavy (mostly RLE with
    short bit-packed stretches) sequences."""
    rng = np.random.default_rng(max_def * 7 + version)
    n = 50_000
    if shape == "random":
        dl = rng.integers(0, max_def + 1, size=n)
    else:
        runs = rng.integers(1, 40, size=n // 8)
        dl = np.repeat(rng.integers(0, max_def + 1, size=runs.size), runs)[:n]
        n = dl.size
    dl = dl.astype(np.uint8)
    vals = rng.integers(-2**40, 2**40, size=int((dl == max_def).sum())).astype(np.int64)
    ch = make(abi.INT64, vals, abi.PLAIN, def_levels=dl, max_def=max_def, version=version, page_rows=6007)
    run_both(decoder, [ch])


@pytest.mark.parametrize("max_def,max_rep", [(1, 0), (2, 0), (3, 1), (7, 0)])
def test_v1_bit_packed_levels(decoder, max_def, max_rep):
    """Deprecated BIT_PACKED (big-endian) level sections of old parquet-mr V1 pages
    (ByteBitPackingValuesReader(maxLevel, BIG_ENDIAN))."""
    rng = np.random.default_rng(max_def * 10 + max_rep)
    n = 30_000
    dl = rng.integers(0, max_def + 1, size=n).astype(np.uint8)
    rl = None
    if max_rep:
        rl = (rng.random(n) < 0.6).astype(np.uint8) * max_rep
        rl[0] = 0
    vals = rng.integers(-2**40, 2**40, size=int((dl == max_def).sum())).astype(np.int64)
    ch = make(abi.INT64, vals, abi.PLAIN, def_levels=dl, rep_levels=rl, max_def=max_def, max_rep=max_rep, version=1,
              level_encoding=abi.BIT_PACKED, page_rows=7000)
    run_both(decoder, [ch])
