"""GPU parity for BYTE_ARRAY (PLAIN, dictionary, DELTA_LENGTH_BYTE_ARRAY), BYTE_STREAM_SPLIT and
FIXED_LEN_BYTE_ARRAY / INT96 dictionaries: libpqgpu.so through the C ABI vs the oracle, bit-exact
(values, offsets, levels, first error)."""
import os

import numpy as np
import pytest

from oracle import pqref
from pqgpu import abi
from tools.synth import writer

from helpers import make, nulls, zipf_dict_column
from test_gpu_parity import assert_same, run_both

pytestmark = pytest.mark.gpu


def _strings(n, seed, lo=0, hi=32, alphabet=b"abcdefghijklmnopqrstuvwxyz0123456789"):
    rng = np.random.default_rng(seed)
    a = np.frombuffer(alphabet, dtype=np.uint8)
    return [a[rng.integers(0, a.size, size=rng.integers(lo, hi + 1))].tobytes() for _ in range(n)]


def _binary_vals(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "ascii":
        return _strings(n, seed, 4, 32)
    if kind == "empty":      # zero-length values: every length prefix is 00 00 00 00
        return [b""] * n
    if kind == "zeros":      # value bytes that look like small lengths: many false candidates
        return [bytes(int(x)) for x in rng.integers(0, 12, size=n)]
    if kind == "smallints":  # little-endian small ints as values
        return [int(x).to_bytes(4, "little") for x in rng.integers(0, 64, size=n)]
    if kind == "random":
        return [rng.integers(0, 256, size=rng.integers(0, 40), dtype=np.uint8).tobytes() for _ in range(n)]
    if kind == "long":       # values longer than the walker's 1 KiB window
        return [rng.integers(0, 256, size=rng.integers(0, 3000), dtype=np.uint8).tobytes() for _ in range(n)]
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["ascii", "empty", "zeros", "smallints", "random", "long"])
@pytest.mark.parametrize("enc", [abi.PLAIN, abi.DELTA_LENGTH_BYTE_ARRAY, abi.RLE_DICTIONARY])
def test_binary_required(decoder, kind, enc):
    n = 600 if kind == "long" else 30_000
    vals = _binary_vals(kind, n, seed=len(kind))
    if enc == abi.RLE_DICTIONARY:  # few distinct values
        vals = [vals[i] for i in np.random.default_rng(1).integers(0, min(len(vals), 400), size=len(vals))]
    run_both(decoder, [make(abi.BYTE_ARRAY, vals, enc, page_rows=7000)])


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("enc", [abi.PLAIN, abi.DELTA_LENGTH_BYTE_ARRAY, abi.PLAIN_DICTIONARY])
@pytest.mark.parametrize("null_frac", [0.0, 0.3, 1.0])
def test_binary_optional(decoder, version, enc, null_frac):
    dl = nulls(20_000, null_frac, seed=3)
    vals = _strings(int(dl.sum()), seed=4, lo=0, hi=48)
    if enc == abi.PLAIN_DICTIONARY:
        vals = [vals[i % 97] for i in range(len(vals))]
    run_both(decoder, [make(abi.BYTE_ARRAY, vals, enc, def_levels=dl, max_def=1, version=version, page_rows=6000,
                            dict_page_encoding=abi.PLAIN_DICTIONARY)])


def test_binary_many_columns_one_batch(decoder):
    chunks = [make(abi.BYTE_ARRAY, _strings(9000, s), e, page_rows=2500)
              for s, e in enumerate([abi.PLAIN, abi.DELTA_LENGTH_BYTE_ARRAY, abi.RLE_DICTIONARY, abi.PLAIN])]
    chunks.append(make(abi.INT64, zipf_dict_column(9000, card=50, seed=1), abi.RLE_DICTIONARY))
    run_both(decoder, chunks)


@pytest.mark.parametrize("dict_entries,lo,hi", [(3, 1, 1), (7, 3, 7), (60, 0, 40), (330, 16, 32), (500, 10, 30)])
def test_binary_dictionary_direct(decoder, dict_entries, lo, hi):
    """Required dictionary-encoded BYTE_ARRAY columns: short entries (C4's flags and modes) take the
    offset scan's direct path (ids -> lengths -> offsets and bytes), dictionaries past its 8 KiB
    staging (330 / 500 entries) the per-value path; several pages and scan blocks, empty entries."""
    words = _strings(dict_entries, seed=dict_entries, lo=lo, hi=hi)
    ids = np.random.default_rng(dict_entries).integers(0, dict_entries, size=50_000)
    run_both(decoder, [make(abi.BYTE_ARRAY, [words[i] for i in ids], abi.RLE_DICTIONARY, page_rows=7000),
                       make(abi.BYTE_ARRAY, [words[i] for i in ids[:9000]], abi.RLE_DICTIONARY, page_rows=3000)])


def test_binary_dictionary_expands_past_estimate(decoder):
    """A dictionary of long entries: the decoded bytes exceed the first byte-buffer estimate,
    the status reports the size needed and decode() retries."""
    words = [bytes([65 + i]) * 5000 for i in range(4)]
    vals = [words[i % 4] for i in range(4000)]
    batch, ref, dcols = run_both(decoder, [make(abi.BYTE_ARRAY, vals, abi.RLE_DICTIONARY)])
    assert dcols[0].binary_data.numel() >= 4000 * 5000


def _err_case(which):
    if which == "plain_eof":      # a value's length runs past the page (EOF at that value)
        ch = make(abi.BYTE_ARRAY, _strings(3000, 1), abi.PLAIN, page_rows=1000)
        ch.pages[1].body = ch.pages[1].body[:-3]
    elif which == "plain_negative":  # slice(negative)
        ch = make(abi.BYTE_ARRAY, _strings(3000, 2), abi.PLAIN, page_rows=1000)
        b = bytearray(ch.pages[2].body)
        b[0:4] = (0xFFFFFFF0).to_bytes(4, "little")
        ch.pages[2].body = bytes(b)
    elif which == "dlba_eof":     # DELTA_LENGTH: value bytes missing at the end
        ch = make(abi.BYTE_ARRAY, _strings(3000, 3), abi.DELTA_LENGTH_BYTE_ARRAY, page_rows=1000)
        ch.pages[0].body = ch.pages[0].body[:-10]
    elif which == "dict_short":   # dictionary page shorter than its entries (PlainBinaryDictionary ctor)
        ch = make(abi.BYTE_ARRAY, _strings(3000, 4), abi.RLE_DICTIONARY, page_rows=1000)
        ch.dict_page = ch.dict_page[:-5]
    elif which == "dict_id":      # dictionary id out of range
        ch = make(abi.BYTE_ARRAY, _strings(3000, 5, 1, 3), abi.RLE_DICTIONARY, page_rows=1000)
        ch.dict_num_values = 3
    return ch


@pytest.mark.parametrize("which", ["plain_eof", "plain_negative", "dlba_eof", "dict_short", "dict_id"])
def test_binary_errors(decoder, which):
    run_both(decoder, [_err_case(which)], expect_error=True)


@pytest.mark.parametrize("k", [0, 1, 700, 4095, 9999])
def test_dlba_negative_length(decoder, k):
    """A negative DELTA_LENGTH_BYTE_ARRAY length (in.slice(negative) in readBytes): CORRUPT at its index, the
    values before it decoded — in the first value, inside and at the end of a 512-length expansion step, and
    in the page's last value (the length stream's steps take the segment expansion, whose stores check
    every length of a step that holds a negative one)."""
    vals = _strings(10_000, 11, 1, 20)
    ch = make(abi.BYTE_ARRAY, vals, abi.DELTA_LENGTH_BYTE_ARRAY, page_rows=10_000)
    lens = np.array([len(v) for v in vals], dtype=np.int32)
    lens[k] = -5
    ch.pages[0].body = writer.delta_encode(lens, abi.INT32) + b"".join(vals)
    run_both(decoder, [ch], expect_error=True)


@pytest.mark.parametrize("case", ["ascii", "empty", "zeros", "smallints", "random", "long", "optional",
                                  "plain_eof", "plain_negative"])
def test_binary_plain_per_page(decoder, per_page_dispatch, case):
    """The one-wave-per-page one-pass PLAIN kernel (k_bin_plain_pg, normally for plans with 4,096 or
    more PLAIN pages) on small plans through the PQG_DISPATCH_PLAIN_ONE_PASS = 3 override: every value
    distribution (false candidates, values longer than a tile, empty values), nulls, and the errors."""
    if case in ("plain_eof", "plain_negative"):
        run_both(decoder, [_err_case(case)], expect_error=True)
    elif case == "optional":
        dl = nulls(20_000, 0.3, seed=3)
        vals = _strings(int(dl.sum()), seed=4, lo=0, hi=48)
        run_both(decoder, [make(abi.BYTE_ARRAY, vals, abi.PLAIN, def_levels=dl, max_def=1, version=2, page_rows=6000)])
    else:
        n = 600 if case == "long" else 30_000
        run_both(decoder, [make(abi.BYTE_ARRAY, _binary_vals(case, n, seed=len(case)), abi.PLAIN, page_rows=7000)])


@pytest.mark.parametrize("ptype,tl", [(abi.FLOAT, 0), (abi.DOUBLE, 0), (abi.INT32, 0), (abi.INT64, 0),
                                      (abi.FIXED_LEN_BYTE_ARRAY, 3), (abi.FIXED_LEN_BYTE_ARRAY, 16)])
@pytest.mark.parametrize("null_frac", [0.0, 0.2])
def test_byte_stream_split(decoder, ptype, tl, null_frac):
    rng = np.random.default_rng(tl + 1)
    dl = nulls(30_001, null_frac, seed=9)
    n = int(dl.sum())
    if ptype == abi.FIXED_LEN_BYTE_ARRAY:
        vals = [rng.integers(0, 256, size=tl, dtype=np.uint8).tobytes() for _ in range(n)]
    else:
        dt = abi.numpy_dtype(ptype)
        vals = rng.integers(0, 256, size=n * dt.itemsize, dtype=np.uint8).view(dt)
    run_both(decoder, [make(ptype, vals, abi.BYTE_STREAM_SPLIT, def_levels=dl, max_def=1, type_length=tl,
                            page_rows=7001)])


def test_byte_stream_split_errors(decoder):
    ch = make(abi.FLOAT, np.arange(3000, dtype=np.float32), abi.BYTE_STREAM_SPLIT, page_rows=1000)
    ch.pages[1].body = ch.pages[1].body[:-1]   # length not a multiple of 4
    run_both(decoder, [ch], expect_error=True)
    ch = make(abi.DOUBLE, np.arange(3000, dtype=np.float64), abi.BYTE_STREAM_SPLIT, page_rows=1000)
    ch.pages[2].body = ch.pages[2].body[:-16]  # fewer encoded values than the page reads
    run_both(decoder, [ch], expect_error=True)


@pytest.mark.parametrize("ptype,tl", [(abi.FIXED_LEN_BYTE_ARRAY, 16), (abi.FIXED_LEN_BYTE_ARRAY, 5),
                                      (abi.FIXED_LEN_BYTE_ARRAY, 8), (abi.INT96, 0)])
def test_fixed_len_dictionary(decoder, ptype, tl):
    rng = np.random.default_rng(tl)
    w = abi.elem_width(ptype, tl)
    words = [rng.integers(0, 256, size=w, dtype=np.uint8).tobytes() for _ in range(300)]
    runs = np.minimum(rng.zipf(1.5, size=20000), 500)
    ids = np.repeat(rng.integers(0, 300, size=runs.size), runs)[:20000]
    run_both(decoder, [make(ptype, [words[i] for i in ids], abi.RLE_DICTIONARY, type_length=tl, page_rows=6000)])


def test_host_path_binary(decoder):
    """pqg_decode_host with BYTE_ARRAY columns (offsets + bytes back in host memory), including
    a dictionary column that needs more bytes than the first estimate."""
    words = [bytes([97 + i % 26]) * (100 + i) for i in range(50)]
    chunks = [make(abi.BYTE_ARRAY, _strings(20000, 7), abi.PLAIN),
              make(abi.BYTE_ARRAY, [words[i % 50] for i in range(20000)], abi.RLE_DICTIONARY)]
    batch = writer.build_batch(chunks)
    ref = pqref.decode_batch(batch, binary_capacity=1 << 23)
    rc, st, res, counts = decoder.decode_host(batch)
    assert rc == 0, st.message
    for i in range(2):
        assert res[i]["values"] == ref.columns[i]["values"]


def test_staged_path_equals_host_path(decoder):
    """The staged host path (library-owned pinned input / output: what the JNI glue uses so that no
    Java array is held across device work) returns what pqg_decode_host returns: BYTE_ARRAY PLAIN and
    an expanding dictionary column, an optional int64 DELTA column with levels, and a nested column;
    then a batch with a value error gives the same status and per-page errors on both paths."""
    words = [bytes([97 + i % 26]) * (100 + i) for i in range(50)]
    dl = nulls(30000, 0.2, seed=4)
    walk = np.cumsum(np.random.default_rng(5).integers(-9, 99, size=int(dl.sum()))).astype(np.int64)
    rng = np.random.default_rng(6)
    rl = (rng.random(25000) < 0.7).astype(np.uint8)
    rl[0] = 0
    dl2 = np.where(rng.random(25000) < 0.1, 1, 2).astype(np.uint8)
    chunks = [make(abi.BYTE_ARRAY, _strings(20000, 7), abi.PLAIN),
              make(abi.BYTE_ARRAY, [words[i % 50] for i in range(20000)], abi.RLE_DICTIONARY),
              make(abi.INT64, walk, abi.DELTA_BINARY_PACKED, def_levels=dl, max_def=1, version=2, page_rows=7000),
              make(abi.DOUBLE, rng.standard_normal(int((dl2 == 2).sum())), abi.PLAIN, def_levels=dl2, rep_levels=rl,
                   max_def=2, max_rep=1, page_rows=6000)]
    batch = writer.build_batch(chunks)
    rc, st, res, counts = decoder.decode_host(batch)
    assert rc == 0, st.message
    rc2, st2, res2, counts2 = decoder.decode_staged(batch)
    assert rc2 == 0, st2.message
    assert np.array_equal(counts, counts2)
    for a, b, cd in zip(res, res2, batch.columns):
        assert a["n_values"] == b["n_values"]
        if cd["physical_type"] == abi.BYTE_ARRAY:
            assert a["values"] == b["values"] and np.array_equal(a["offsets"], b["offsets"])
        else:
            assert np.array_equal(np.asarray(a["values"]).view(np.uint8), np.asarray(b["values"]).view(np.uint8))
        for k in ("def_levels", "rep_levels"):
            assert (a[k] is None) == (b[k] is None) and (a[k] is None or np.array_equal(a[k], b[k]))
    # an invalid dictionary id in the dictionary column's second page: same status, same page errors
    vals = np.random.default_rng(9).integers(0, 40, size=30000).astype(np.int64)
    bad = make(abi.INT64, vals, abi.RLE_DICTIONARY, page_rows=10000)
    bad.dict_num_values = 35
    ids, _ = writer.dictionary_encode(vals)
    first_bad = int(np.argmax(ids >= 35))
    batch = writer.build_batch([chunks[2], bad])
    rc, st, _, _ = decoder.decode_host(batch)
    pe = decoder.page_errors(batch.n_pages)
    rc2, st2, _, _ = decoder.decode_staged(batch)
    pe2 = decoder.page_errors(batch.n_pages)
    assert rc == rc2 == abi.ERR_DICT_ID and (st.page, st.value_index) == (st2.page, st2.value_index)
    assert pe == pe2
    bad_pages = [p for p, e in enumerate(pe) if e[0]]
    col_pages = [p for p in range(batch.n_pages) if batch.pages[p]["column"] == 1]
    assert bad_pages[0] == col_pages[first_bad // 10000]
    assert pe[bad_pages[0]] == (abi.ERR_DICT_ID, abi.PHASE_VALUE, first_bad % 10000)
    assert all(pe[p][0] == 0 for p in range(batch.n_pages) if batch.pages[p]["column"] == 0)


# ---- DELTA_BYTE_ARRAY (DeltaByteArrayReader) -----------------------------------------------------------------

def _dba_vals(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "urls":      # sorted keys sharing long prefixes (the encoding's use case)
        return sorted(f"https://example.org/{rng.integers(0, 50)}/item/{rng.integers(0, 10**6):07d}".encode()
                      for _ in range(n))
    if kind == "random":
        return _strings(n, seed, 0, 24, alphabet=b"ab")
    if kind == "long":      # values past the kernel's 2 KiB LDS value buffer, with shared prefixes
        base = rng.integers(97, 123, size=6000, dtype=np.uint8).tobytes()
        return [base[:rng.integers(0, 6000)] + bytes([97 + i % 26]) * int(rng.integers(0, 40)) for i in range(n)]
    if kind == "growing":   # prefix i + 1 of value i + 1 = all of value i
        return [b"x" * i for i in range(n)]
    raise ValueError(kind)


@pytest.mark.parametrize("kind,n", [("urls", 30000), ("random", 30000), ("long", 400), ("growing", 700)])
def test_delta_byte_array(decoder, kind, n):
    run_both(decoder, [make(abi.BYTE_ARRAY, _dba_vals(kind, n, 5), abi.DELTA_BYTE_ARRAY, page_rows=5000)])


def test_delta_byte_array_long_pages(decoder):
    # pages of more than 256 chunks of 256 values: the serial chain (k_dba_chain) beside the per-chunk one
    vals = _dba_vals("urls", 150_000, 9)
    run_both(decoder, [make(abi.BYTE_ARRAY, vals, abi.DELTA_BYTE_ARRAY, page_rows=70_000)])


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("null_frac", [0.2, 1.0])
def test_delta_byte_array_optional(decoder, version, null_frac):
    dl = nulls(20_000, null_frac, seed=8)
    vals = _dba_vals("urls", int(dl.sum()), 6)
    run_both(decoder, [make(abi.BYTE_ARRAY, vals, abi.DELTA_BYTE_ARRAY, def_levels=dl, max_def=1, version=version,
                            page_rows=6000)])


def _dba_err(which):
    from tools.synth import writer as W
    if which == "prefix_too_long":   # prefix > previous.length (arraycopy IndexOutOfBounds)
        body = W.delta_encode(np.array([0, 9], dtype=np.int32), abi.INT32) + W.dlba_encode([b"abc", b"x"])
    elif which == "suffix_short":    # suffix bytes missing: "Failed to read N bytes"
        body = W.dba_encode([b"abcdef", b"abcxyz", b"q"])[:-2]
    elif which == "negative_suffix":  # slice(negative)
        body = W.delta_encode(np.array([0, 0], dtype=np.int32), abi.INT32) + \
            W.delta_encode(np.array([2, -5], dtype=np.int32), abi.INT32) + b"ab"
    elif which == "prefix_stream_short":  # fewer prefix lengths than values: DELTA_PAST_END
        body = W.delta_encode(np.array([0], dtype=np.int32), abi.INT32) + W.dlba_encode([b"abc", b"de"])
    ch = make(abi.BYTE_ARRAY, [b"a", b"b"] if which != "suffix_short" else [b"a", b"b", b"c"], abi.DELTA_BYTE_ARRAY)
    ch.pages[0].body = body
    return ch


@pytest.mark.parametrize("which", ["prefix_too_long", "suffix_short", "negative_suffix", "prefix_stream_short"])
def test_delta_byte_array_errors(decoder, which):
    run_both(decoder, [_dba_err(which)], expect_error=True)


def test_delta_byte_array_mixed_pages(decoder):
    """One chunk of pages whose values stay under the 2 KiB LDS value buffer (chunk-parallel copy:
    tails, chain of chunk tails, chunks) next to pages with longer values (serial copy)."""
    short = [b"x" * (i % 1900) + bytes([97 + i % 26]) for i in range(3000)]
    grow = [b"y" * min(i * 3, 2600) for i in range(1200)]
    run_both(decoder, [make(abi.BYTE_ARRAY, short + grow + short, abi.DELTA_BYTE_ARRAY, page_rows=1700)])


@pytest.mark.parametrize("at", [300, 1000, 1279])
def test_delta_byte_array_error_mid_page(decoder, at):
    """An invalid prefix length (longer than the previous value) inside a page of several
    256-value chunks: values before it decode, the error is reported at its index."""
    from tools.synth import writer as W
    vals = _dba_vals("urls", 1280, 9)
    pre = [0] + [len(os.path.commonprefix([vals[i - 1], vals[i]])) for i in range(1, len(vals))]
    pre[at] = len(vals[at - 1]) + 5
    suf = [v[min(p, len(v)):] for v, p in zip(vals, pre)]
    ch = make(abi.BYTE_ARRAY, vals, abi.DELTA_BYTE_ARRAY)
    ch.pages[0].body = W.delta_encode(np.array(pre, dtype=np.int32), abi.INT32) + W.dlba_encode(suf)
    run_both(decoder, [ch], expect_error=True)


# ---- PLAIN BYTE_ARRAY pages walked in 16 KiB segments (k_bin_walk_seg: plans with few such pages) ----

@pytest.mark.parametrize("kind", ["ascii", "empty", "zeros", "smallints", "random", "long"])
@pytest.mark.parametrize("version", [1, 2])
def test_binary_plain_segmented(decoder, kind, version):
    """Pages of 100-900 KB (many segments each): every kind of value bytes, including ones whose
    bytes read as small lengths (the speculative segment starts then fail and are walked again), and
    nullable V1 / V2 pages (the data section starts after the levels, at any alignment)."""
    n = 2000 if kind == "long" else 60_000
    vals = _binary_vals(kind, n, seed=11 + len(kind))
    dl = nulls(n + n // 9, 0.1, seed=5)
    vals = vals[: int(dl.sum())]
    run_both(decoder, [make(abi.BYTE_ARRAY, vals, abi.PLAIN, def_levels=dl, max_def=1, version=version,
                            page_rows=len(dl) // 2 + 1)])
    run_both(decoder, [make(abi.BYTE_ARRAY, vals, abi.PLAIN, page_rows=len(vals) // 2 + 3)])


@pytest.mark.parametrize("where", [0.0, 0.1, 0.5, 0.93, 0.999])
@pytest.mark.parametrize("how", ["negative", "overrun", "truncate"])
def test_binary_plain_segmented_errors(decoder, where, how):
    """An error at any point of a large page (in its first, a middle or the last segment): the
    status equals the oracle's (page, value index, code); nothing past the error is required."""
    vals = _strings(30_000, 7, 0, 40)
    ch = make(abi.BYTE_ARRAY, vals, abi.PLAIN, page_rows=30_000)
    body = bytearray(ch.pages[0].body)
    k = int(where * (len(vals) - 1))
    pos = sum(4 + len(v) for v in vals[:k])
    if how == "negative":
        body[pos:pos + 4] = (0x80000001).to_bytes(4, "little")
    elif how == "overrun":
        body[pos:pos + 4] = (len(body) * 2).to_bytes(4, "little")
    else:
        body = body[:pos + 2]
    ch.pages[0].body = bytes(body)
    run_both(decoder, [ch], expect_error=True)


def test_binary_plain_segmented_trailing_bytes(decoder):
    """A page whose header counts fewer values than its bytes hold: the walk stops at the count
    (the rest is never read, garbage included), in whichever segment the count ends."""
    vals = _strings(40_000, 8, 0, 30)
    ch = make(abi.BYTE_ARRAY, vals, abi.PLAIN, page_rows=40_000)
    ch.pages[0].body = ch.pages[0].body + bytes(np.random.default_rng(1).integers(0, 256, 50_000, dtype=np.uint8))
    for nv in (1, 777, 23_456, 40_000):
        ch.pages[0].num_values = nv
        ch.values = vals[:nv]
        run_both(decoder, [ch])


# ---- PLAIN-only BYTE_ARRAY columns in one pass (k_bin_bases + k_bin_plain, 2 KiB tiles) ----

def _plan_both(decoder, chunks):
    """Decode through a plan (two launches) and compare with the oracle after each; returns the plan."""
    batch = writer.build_batch(chunks)
    ref = pqref.decode_batch(batch)
    assert ref.code == 0, ref.status
    plan = decoder.plan(decoder.upload(batch))
    for _ in range(2):
        plan.launch()
        rc, st = plan.sync()
        assert rc == 0, st.message
        for i, cd in enumerate(batch.columns):
            col = plan.columns[i]
            n = ref.columns[i]["n_values"]
            assert_same(col.numpy(), ref.columns[i]["values"], cd["physical_type"])
            if cd["physical_type"] == abi.BYTE_ARRAY:
                assert np.array_equal(col.offsets().cpu().numpy()[: n + 1], ref.columns[i]["offsets"][: n + 1])
    return plan


@pytest.fixture(params=["tiles", "pages"])
def one_pass_kernel(request, decoder):
    """The one-pass PLAIN kernel a small plan takes: the tiles (default) or one wave per page (the
    PQG_DISPATCH_PLAIN_ONE_PASS = 3 override; plans with 4,096 or more PLAIN pages take it by default)."""
    if request.param == "pages":
        decoder.set_dispatch(abi.DISPATCH_PLAIN_ONE_PASS, 3)
    yield request.param
    decoder.set_dispatch(abi.DISPATCH_PLAIN_ONE_PASS, 2)


@pytest.fixture
def per_page_dispatch(decoder):
    decoder.set_dispatch(abi.DISPATCH_PLAIN_ONE_PASS, 3)
    yield
    decoder.set_dispatch(abi.DISPATCH_PLAIN_ONE_PASS, 2)


def test_binary_plain_one_pass_no_fallback(decoder, one_pass_kernel):
    """Well-formed PLAIN pages take the one-pass path and never fall back; mixed with a column whose
    pages are dictionary-encoded (per-value path) in the same plan."""
    a = make(abi.BYTE_ARRAY, _strings(50_000, 21, 0, 60), abi.PLAIN, page_rows=9000)
    b = make(abi.BYTE_ARRAY, [_strings(300, 22)[i % 300] for i in range(20_000)], abi.RLE_DICTIONARY, page_rows=7000)
    plan = _plan_both(decoder, [a, b])
    assert plan.plain_fallbacks == 0


def test_binary_plain_one_pass_fallback(decoder, one_pass_kernel):
    """Bytes after a page's values (the reader ignores them): the plan falls back to the per-value path
    once and keeps it; the result equals the oracle on both launches."""
    vals = _strings(20_000, 23, 0, 30)
    ch = make(abi.BYTE_ARRAY, vals, abi.PLAIN, page_rows=10_000)
    ch.pages[0].body = ch.pages[0].body + b"\x07\x00\x00\x00abcdefg" + bytes(300)
    plan = _plan_both(decoder, [ch])
    assert plan.plain_fallbacks == 1


def test_binary_plain_fallback_two_plans_one_sync(decoder, one_pass_kernel):
    """pqg_sync checks and repairs every plan launched since the previous sync, not only the last
    one: plan A (a page with bytes after its values) and plan B launched back to back, one sync."""
    vals = _strings(20_000, 23, 0, 30)
    a = make(abi.BYTE_ARRAY, vals, abi.PLAIN, page_rows=10_000)
    a.pages[0].body = a.pages[0].body + b"\x07\x00\x00\x00abcdefg" + bytes(300)
    b = make(abi.BYTE_ARRAY, _strings(30_000, 24, 0, 40), abi.PLAIN, page_rows=8000)
    batches = [writer.build_batch([a]), writer.build_batch([b])]
    refs = [pqref.decode_batch(x) for x in batches]
    plans = [decoder.plan(decoder.upload(x)) for x in batches]
    for p in plans:
        p.launch()
    rc, st = plans[1].sync()
    assert rc == 0, st.message
    for p, ref in zip(plans, refs):
        n = ref.columns[0]["n_values"]
        assert np.array_equal(p.columns[0].offsets().cpu().numpy()[: n + 1], ref.columns[0]["offsets"][: n + 1])
        assert_same(p.columns[0].numpy(), ref.columns[0]["values"], abi.BYTE_ARRAY)
    assert plans[0].plain_fallbacks == 1 and plans[1].plain_fallbacks == 0
    for p in plans:
        p.close()


@pytest.mark.parametrize("lens", ["tile_sized", "tile_minus_4", "spanning", "empty_then_long"])
def test_binary_plain_tile_edges(decoder, lens, one_pass_kernel):
    """Values whose boundaries fall on 2 KiB tile edges, values longer than two tiles (a tile with no
    value start; bytes past the staged tiles), and runs of empty values."""
    rng = np.random.default_rng(len(lens))
    if lens == "tile_sized":
        vals = [bytes(rng.integers(0, 256, 2044, dtype=np.uint8)) for _ in range(40)]
    elif lens == "tile_minus_4":
        vals = [bytes(rng.integers(0, 256, int(x), dtype=np.uint8)) for x in rng.integers(2040, 2050, 60)]
    elif lens == "spanning":
        vals = [bytes(rng.integers(0, 256, int(x), dtype=np.uint8)) for x in rng.integers(0, 9000, 80)]
    else:
        vals = ([b""] * 3000 + [bytes(5000)] + [b"x"] * 700) * 3
    run_both(decoder, [make(abi.BYTE_ARRAY, vals, abi.PLAIN, page_rows=len(vals) // 3 + 1)])
    dl = nulls(len(vals) + 50, 0.05, seed=2)
    nn = int(dl.sum())
    run_both(decoder, [make(abi.BYTE_ARRAY, (vals * (nn // len(vals) + 1))[:nn], abi.PLAIN, def_levels=dl, max_def=1,
                            version=1, page_rows=len(dl) // 2 + 1)])


# ---- dictionary-direct BYTE_ARRAY columns (launch_dict_dd: walk + chunk byte sums, per-column scan,
# offsets and value bytes from the ids in registers) ------------------------------------------------------

def _lineitem_words():
    return [b"DELIVER IN PERSON", b"COLLECT COD", b"NONE", b"TAKE BACK RETURN", b"R", b"A", b"N", b"", b"AIR"]


@pytest.fixture(params=[1, 0], ids=["fused", "split"])
def dict_fused(decoder, request):
    """PQG_DISPATCH_DICT_FUSED: 1 = walk + expansion in one launch (k_dict_fused_dd), 0 = the split
    launches (k_dict_runs + k_dict_tiles_dd), which are also the timeout re-run of the fused one."""
    decoder.set_dispatch(abi.DISPATCH_DICT_FUSED, request.param)
    yield request.param
    decoder.set_dispatch(abi.DISPATCH_DICT_FUSED, 1)


@pytest.mark.parametrize("dict_direct", [1, 0])
def test_dictionary_direct_interleaved_columns(decoder, dict_direct, dict_fused):
    """Several dictionary-direct columns whose pages are interleaved in the page table (the plan sorts
    their chunks by column and pads each column to whole workgroups), beside a column of another kind;
    PQG_DISPATCH_DICT_DIRECT = 0 sends the same columns through ids -> map -> copy: equal results."""
    words = _lineitem_words()
    rng = np.random.default_rng(17)
    chunks = []
    for k, (n, card, rows) in enumerate([(47_000, 3, 20000), (30_001, 9, 7000), (8_191, 2, 1000), (25_000, 7, 4096)]):
        w = words[k: k + card] if k + card <= len(words) else words[:card]
        ids = rng.integers(0, card, size=n)
        chunks.append(make(abi.BYTE_ARRAY, [w[i] for i in ids], abi.RLE_DICTIONARY, page_rows=rows))
    chunks.append(make(abi.INT64, zipf_dict_column(20_000, card=40, seed=5), abi.RLE_DICTIONARY, page_rows=3000))
    batch = writer.build_batch(chunks)
    order = np.argsort(np.arange(batch.n_pages) % 5, kind="stable")
    cols = batch.pages["column"][order]
    for c in range(len(chunks)):  # keep each column's page order
        idx = np.nonzero(cols == c)[0]
        order[idx] = np.sort(order[idx])
    batch.pages = batch.pages[order]
    batch.page_slot_offsets = batch.page_slot_offsets[order]
    ref = pqref.decode_batch(batch)
    assert ref.code == 0
    decoder.set_dispatch(abi.DISPATCH_DICT_DIRECT, dict_direct)
    try:
        dcols, st = decoder.decode(decoder.upload(batch), check=False)
    finally:
        decoder.set_dispatch(abi.DISPATCH_DICT_DIRECT, 1)
    assert st.code == 0, st.message
    for i, cd in enumerate(batch.columns):
        assert_same(dcols[i].numpy(), ref.columns[i]["values"], cd["physical_type"])
        if cd["physical_type"] == abi.BYTE_ARRAY:
            n = ref.columns[i]["n_values"]
            assert np.array_equal(dcols[i].offsets().cpu().numpy(), ref.columns[i]["offsets"][: n + 1])


@pytest.mark.parametrize("lens", [(0, 0), (1, 4000), (2000, 2000, 2000), (0, 1, 23, 24, 64),
                                  (2, 3), (0, 2, 17, 32), (17, 11, 4, 16), (7, 3, 4, 4, 5, 4, 3), (16,), (32, 32, 1)])
def test_dictionary_direct_entry_lengths(decoder, lens, dict_fused):
    """Entry lengths around the kernel's byte paths: empty entries only, 1-byte entries, entries of 2..32
    bytes (composed into whole 16-byte output blocks: C4's ship instruct / mode shapes, blocks that start
    inside, at the start of and between entries, 16-byte entries, empty entries between), longer ones
    (written value by value), and mixes in one chunk."""
    rng = np.random.default_rng(len(lens))
    words = [bytes(rng.integers(65, 91, size=n, dtype=np.uint8)) for n in lens]
    ids = rng.integers(0, len(words), size=9000)
    ids[:600] = 0  # an RLE run of the first entry, then mixed runs
    run_both(decoder, [make(abi.BYTE_ARRAY, [words[i] for i in ids], abi.RLE_DICTIONARY, page_rows=3500)])


def test_dictionary_direct_expands_past_estimate(decoder):
    """A dictionary-direct column whose bytes exceed the first byte-buffer estimate: the byte total
    (k_dd_bases) reports the size needed and decode() retries."""
    words = [bytes([66 + i]) * 2600 for i in range(3)]  # 7.8 KB dictionary page: dictionary-direct
    vals = [words[i % 3] for i in range(6000)]
    batch, ref, dcols = run_both(decoder, [make(abi.BYTE_ARRAY, vals, abi.RLE_DICTIONARY, page_rows=2000)])
    assert dcols[0].binary_data.numel() >= 6000 * 2600


def test_dictionary_direct_error_stays_in_its_column(decoder):
    """An id past the dictionary in one dictionary-direct column: the oracle's status, and the other
    dictionary-direct column of the batch decodes completely."""
    words = _lineitem_words()
    rng = np.random.default_rng(23)
    good_ids = rng.integers(0, 7, size=30_000)
    good = make(abi.BYTE_ARRAY, [words[i] for i in good_ids], abi.RLE_DICTIONARY, page_rows=9000)
    bad = make(abi.BYTE_ARRAY, [words[i] for i in rng.integers(0, 6, size=30_000)], abi.RLE_DICTIONARY,
               page_rows=9000)
    bad.dict_num_values = 4
    batch = writer.build_batch([bad, good])
    ref = pqref.decode_batch(batch)
    dcols, st = decoder.decode(decoder.upload(batch), check=False)
    assert ref.code != 0 and (int(st.code), int(st.page), int(st.value_index)) == ref.status
    assert_same(dcols[1].numpy(), [words[i] for i in good_ids], abi.BYTE_ARRAY)


def test_dictionary_direct_plan_relaunch(decoder, dict_fused):
    """A plan launched twice: the chunk sums and bases are rewritten per launch (nothing stale)."""
    words = _lineitem_words()
    ids = np.random.default_rng(29).integers(0, 9, size=40_000)
    _plan_both(decoder, [make(abi.BYTE_ARRAY, [words[i] for i in ids], abi.RLE_DICTIONARY, page_rows=20000),
                         make(abi.BYTE_ARRAY, [words[i] for i in ids[::-1]], abi.RLE_DICTIONARY, page_rows=6000)])


@pytest.mark.parametrize("short", [0.5, 0.9])
def test_dictionary_direct_short_buffer_keeps_prefix(decoder, short):
    """A byte buffer shorter than the column: the call reports the size needed and the bytes below the
    capacity are the column's (entries of 2..32 bytes: the block gather, whose partial last block of a
    tile is carried into the next tile; a next tile past the capacity stores it byte-wise)."""
    rng = np.random.default_rng(int(short * 10))
    words = _strings(40, seed=31, lo=2, hi=31)
    ids = rng.integers(0, len(words), size=60_000)
    batch = writer.build_batch([make(abi.BYTE_ARRAY, [words[i] for i in ids], abi.RLE_DICTIONARY, page_rows=20000)])
    ref = pqref.decode_batch(batch)
    assert ref.code == 0
    want = b"".join(ref.columns[0]["values"])
    cols = decoder.alloc_columns(batch)
    cap = int(len(want) * short) + 5
    import torch
    cols[0].binary_data = torch.zeros(cap, dtype=torch.uint8, device=decoder.device)
    rc, st, _ = decoder._decode_once(decoder.upload(batch), cols, None)
    assert rc == abi.ERR_INVALID_ARG and st.message.startswith(b"binary capacity"), st.message
    assert int(st.value_index) >= len(want)
    got = cols[0].binary_data.cpu().numpy().tobytes()
    assert got == want[:cap]


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("null_frac", [0.0, 0.1, 0.6, 1.0])
def test_dictionary_direct_optional(decoder, version, null_frac, dict_fused):
    """Optional dictionary BYTE_ARRAY columns take the dictionary-direct path too (round 6): the walk reads
    each page's n_values ids (from k_levels, or the V2 header counts), offsets[n] closes at the column's
    non-null count; all-null pages and all-null columns included."""
    words = _lineitem_words() + _strings(40, seed=77, lo=2, hi=30)
    dl = nulls(30_000, null_frac, seed=int(null_frac * 10) + version)
    n = int(dl.sum())
    ids = np.random.default_rng(version).integers(0, len(words), size=n)
    run_both(decoder, [make(abi.BYTE_ARRAY, [words[i] for i in ids], abi.RLE_DICTIONARY, def_levels=dl, max_def=1,
                            version=version, page_rows=4000),
                       make(abi.INT64, zipf_dict_column(9000, card=30, seed=2), abi.RLE_DICTIONARY, page_rows=3000)])


@pytest.mark.parametrize("version", [1, 2])
def test_dictionary_direct_nested(decoder, version):
    """A repeated dictionary BYTE_ARRAY leaf (rep + def levels; LIST<string>): dictionary-direct, equal to the
    oracle (values, offsets, both level arrays), and equal to the ids -> map -> copy path."""
    rng = np.random.default_rng(5)
    rl, dl = [], []
    for L in rng.poisson(2.5, size=6000):
        if L == 0:
            rl.append(0); dl.append(int(rng.integers(0, 2)))
        for j in range(L):
            rl.append(0 if j == 0 else 1); dl.append(3 if rng.random() >= 0.15 else 2)
    rl = np.array(rl, dtype=np.uint8)
    dl = np.array(dl, dtype=np.uint8)
    words = _strings(300, seed=8, lo=0, hi=24)
    vals = [words[i] for i in rng.integers(0, len(words), size=int((dl == 3).sum()))]
    ch = make(abi.BYTE_ARRAY, vals, abi.RLE_DICTIONARY, def_levels=dl, rep_levels=rl, max_def=3, max_rep=1,
              version=version, page_rows=2500)
    batch, ref, a = run_both(decoder, [ch])
    decoder.set_dispatch(abi.DISPATCH_DICT_DIRECT, 0)
    try:
        _, _, b = run_both(decoder, [ch])
    finally:
        decoder.set_dispatch(abi.DISPATCH_DICT_DIRECT, 1)
    assert np.array_equal(a[0].offsets().cpu().numpy(), b[0].offsets().cpu().numpy())


def test_dictionary_direct_optional_errors(decoder):
    """An id past the dictionary on an optional dictionary-direct column (V1 and V2 pages): the oracle's
    status (page, value index)."""
    words = _lineitem_words()
    dl = nulls(20_000, 0.2, seed=3)
    n = int(dl.sum())
    ids = np.random.default_rng(4).integers(0, 6, size=n)
    for version in (1, 2):
        ch = make(abi.BYTE_ARRAY, [words[i] for i in ids], abi.RLE_DICTIONARY, def_levels=dl, max_def=1,
                  version=version, page_rows=3000)
        ch.dict_num_values = 4
        run_both(decoder, [ch], expect_error=True)


@pytest.mark.parametrize("shape", ["16k", "3000_short", "2000_over_32k", "long_entries", "mixed_long", "65536"])
def test_dictionary_direct_large(decoder, shape, dict_fused):
    """Dictionaries past the LDS staging (over 2,048 entries or 32 KiB; at most 65,536 entries): u16 ids,
    entries and value bytes gathered from HBM (k_dd_gsums / k_dd_gstr); entries over 32 bytes take the byte
    path; equal to the oracle and to the ids -> map -> copy path."""
    card, lo, hi, n = {"16k": (16384, 4, 32, 120_000), "3000_short": (3000, 0, 8, 60_000),
                       "2000_over_32k": (2000, 20, 40, 60_000), "long_entries": (2500, 33, 90, 30_000),
                       "mixed_long": (5000, 0, 48, 50_000), "65536": (65536, 1, 6, 200_000)}[shape]
    words = _strings(card, seed=card, lo=lo, hi=hi)
    rng = np.random.default_rng(card)
    runs = np.minimum(rng.zipf(1.6, size=n), 300)
    ids = np.repeat(rng.integers(0, card, size=runs.size), runs)[:n]
    if shape == "65536":
        ids[:card] = np.arange(card)  # every entry used: the dictionary holds all 65,536
    vals = [words[i] for i in ids]
    batch, ref, a = run_both(decoder, [make(abi.BYTE_ARRAY, vals, abi.RLE_DICTIONARY, page_rows=9000)])
    decoder.set_dispatch(abi.DISPATCH_DICT_DIRECT, 0)
    try:
        _, _, b = run_both(decoder, [make(abi.BYTE_ARRAY, vals, abi.RLE_DICTIONARY, page_rows=9000)])
    finally:
        decoder.set_dispatch(abi.DISPATCH_DICT_DIRECT, 1)
    assert np.array_equal(a[0].offsets().cpu().numpy(), b[0].offsets().cpu().numpy())


@pytest.mark.parametrize("version", [1, 2])
def test_dictionary_direct_large_optional(decoder, version):
    """A nullable column with a 10,000-entry dictionary beside a small-dictionary one (both dictionary-direct
    kinds in one plan), 15 % nulls."""
    words = _strings(10_000, seed=12, lo=1, hi=28)
    small = _lineitem_words()
    dl = nulls(70_000, 0.15, seed=version)
    n = int(dl.sum())
    rng = np.random.default_rng(3)
    run_both(decoder, [make(abi.BYTE_ARRAY, [words[i] for i in rng.integers(0, 10_000, size=n)], abi.RLE_DICTIONARY,
                            def_levels=dl, max_def=1, version=version, page_rows=8000),
                       make(abi.BYTE_ARRAY, [small[i] for i in rng.integers(0, len(small), size=40_000)],
                            abi.RLE_DICTIONARY, page_rows=7000)])


def test_dictionary_direct_large_error(decoder):
    """An id past a large dictionary: the oracle's status."""
    words = _strings(5000, seed=5, lo=2, hi=20)
    ids = np.random.default_rng(9).integers(0, 5000, size=40_000)
    ch = make(abi.BYTE_ARRAY, [words[i] for i in ids], abi.RLE_DICTIONARY, page_rows=6000)
    ch.dict_num_values = 4000
    run_both(decoder, [ch], expect_error=True)


def test_dictionary_direct_large_short_buffer(decoder):
    """A byte buffer shorter than the column (large dictionary): the size needed is reported and the bytes
    below the capacity are the column's."""
    words = _strings(4000, seed=6, lo=2, hi=31)
    ids = np.random.default_rng(10).integers(0, 4000, size=50_000)
    batch = writer.build_batch([make(abi.BYTE_ARRAY, [words[i] for i in ids], abi.RLE_DICTIONARY, page_rows=20000)])
    ref = pqref.decode_batch(batch)
    want = b"".join(ref.columns[0]["values"])
    cols = decoder.alloc_columns(batch)
    cap = len(want) // 2 + 3
    import torch
    cols[0].binary_data = torch.zeros(cap, dtype=torch.uint8, device=decoder.device)
    rc, st, _ = decoder._decode_once(decoder.upload(batch), cols, None)
    assert rc == abi.ERR_INVALID_ARG and int(st.value_index) >= len(want)
    assert cols[0].binary_data.cpu().numpy().tobytes() == want[:cap]


@pytest.mark.parametrize("case", ["ok", "cut", "neg_len", "long_len", "more_declared", "fewer_declared", "huge_entry",
                                  "70k_entries"])
def test_large_dictionary_page_walk(decoder, case):
    """Dictionary pages of 16 KiB or more are walked per 2 KiB tile (k_dent_walk / k_dent_resolve /
    k_dent_scatter): entries, the dictionary's error (PlainBinaryDictionary ctor) and the decoded values equal
    the oracle's — truncated pages, a negative or oversized length in the middle, more or fewer entries
    declared than the page holds, an entry longer than a tile, and a dictionary past 65,536 entries (ids ->
    map -> copy path)."""
    rng = np.random.default_rng(len(case))
    card = 70_000 if case == "70k_entries" else 3000
    words = _strings(card, seed=card, lo=0, hi=20)
    if case == "huge_entry":
        words[5] = bytes(rng.integers(65, 91, size=7000, dtype=np.uint8))
    if case == "70k_entries":  # every entry used: 70,000 distinct values, past the u16 ids
        ids = np.concatenate([np.arange(card), rng.integers(0, card, size=10_000)])
    else:
        ids = rng.integers(0, 2900, size=60_000)
    ch = make(abi.BYTE_ARRAY, [words[i] for i in ids], abi.RLE_DICTIONARY, page_rows=9000)
    d = bytearray(ch.dict_page)
    if case == "cut":
        ch.dict_page = bytes(d[: len(d) - 37])
    elif case in ("neg_len", "long_len"):
        p = 0
        for _ in range(1500):  # the 1,500th entry's length prefix
            p += 4 + int.from_bytes(d[p:p + 4], "little")
        d[p:p + 4] = ((0x80000000 | 5) if case == "neg_len" else len(d) * 3).to_bytes(4, "little")
        ch.dict_page = bytes(d)
    elif case == "more_declared":
        ch.dict_num_values += 2
    elif case == "fewer_declared":
        ch.dict_num_values -= 50  # the page's last entries are never read; ids past them are errors
    batch = writer.build_batch([ch])
    ref = pqref.decode_batch(batch)
    run_both(decoder, [ch], expect_error=ref.code != 0)
