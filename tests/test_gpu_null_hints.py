"""V2 header null counts as a verified hint (PQG_PAGE_NULL_COUNT, PQG_DISPATCH_NULL_HINTS).

The reference reads DataPageV2.getNullCount (parquet-column/.../column/page/DataPageV2.java:197-199) but
decodes by the definition levels: a value is read for every slot with dl == max_def
(ColumnReaderBase.java:650-676, readPageV2 :760-771). The decoder starts its value kernels from the
header counts beside the level kernel, which verifies them; a wrong count (or a level error on such a
page) makes pqg_sync re-run the plan level-first. Whatever the header says, the result and the first
error are the oracle's (which, like the reference, never reads num_nulls)."""
import numpy as np
import pytest
import torch

from oracle import pqref
from pqgpu import abi
from tools.synth import writer

from helpers import assert_same, make, nulls
from test_gpu_parity import run_both



def _strings(n, seed):
    rng = np.random.default_rng(seed)
    a = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", dtype=np.uint8)
    return [a[rng.integers(0, a.size, size=rng.integers(0, 20))].tobytes() for _ in range(n)]


def _c3_like(n_slots=24_000, seed=3, version=2, page_rows=5000):
    """Optional columns of C3's kinds (DELTA int32 / int64, PLAIN double, PLAIN strings) plus an optional
    dictionary int64 and DELTA_LENGTH strings column, 10 % nulls."""
    rng = np.random.default_rng(seed)
    chunks = []
    for k, (ptype, enc) in enumerate([(abi.INT32, abi.DELTA_BINARY_PACKED), (abi.INT64, abi.DELTA_BINARY_PACKED),
                                      (abi.DOUBLE, abi.PLAIN), (abi.BYTE_ARRAY, abi.PLAIN),
                                      (abi.INT64, abi.RLE_DICTIONARY), (abi.BYTE_ARRAY, abi.DELTA_LENGTH_BYTE_ARRAY)]):
        dl = nulls(n_slots, 0.1, seed=seed + k)
        n = int(dl.sum())
        if ptype == abi.BYTE_ARRAY:
            vals = _strings(n, seed + k)
        elif ptype == abi.DOUBLE:
            vals = rng.standard_normal(n)
        elif enc == abi.RLE_DICTIONARY:
            vals = rng.integers(-50, 50, size=n).astype(np.int64) * 1_000_003
        elif ptype == abi.INT64:
            vals = np.cumsum(rng.integers(-1000, 100000, size=n)).astype(np.int64)
        else:
            vals = rng.integers(-2**31, 2**31 - 1, size=n).astype(np.int32)
        chunks.append(make(ptype, vals, enc, def_levels=dl, max_def=1, version=version, page_rows=page_rows))
    return chunks


def _check(batch, ref, cols):
    for i, cd in enumerate(batch.columns):
        n = ref.columns[i]["n_values"]
        assert cols[i].n_values == n
        assert_same(cols[i].numpy(), ref.columns[i]["values"], cd["physical_type"])
        if cd["physical_type"] == abi.BYTE_ARRAY:
            assert np.array_equal(cols[i].offsets().cpu().numpy()[: n + 1], ref.columns[i]["offsets"][: n + 1])
        assert np.array_equal(cols[i].def_levels[: batch.column_slots[i]].cpu().numpy(), ref.columns[i]["def_levels"])


def _plan_run(decoder, batch, launches=2):
    """Launch a plan `launches` times (sync after each), compare with the oracle each time; return the plan."""
    ref = pqref.decode_batch(batch)
    assert ref.code == 0, ref.status
    plan = decoder.plan(decoder.upload(batch))
    for _ in range(launches):
        plan.launch()
        rc, st = plan.sync()
        assert rc == 0, st.message
        for i, cd in enumerate(batch.columns):
            n = ref.columns[i]["n_values"]
            col = plan.columns[i]
            if cd["physical_type"] == abi.BYTE_ARRAY:
                assert np.array_equal(col.offsets().cpu().numpy()[: n + 1], ref.columns[i]["offsets"][: n + 1])
                assert_same(col.numpy(), ref.columns[i]["values"], cd["physical_type"])
            else:
                assert_same(col.typed()[:n].cpu().numpy(), ref.columns[i]["values"], cd["physical_type"])
            assert np.array_equal(col.def_levels[: batch.column_slots[i]].cpu().numpy(), ref.columns[i]["def_levels"])
    return plan


def test_build_batch_sets_the_hint_on_v2_pages():
    """(host) build_batch / the framing carry the V2 header's num_nulls with PQG_PAGE_NULL_COUNT."""
    batch = writer.build_batch(_c3_like(n_slots=3000, page_rows=1000))
    assert (batch.pages["flags"] & abi.PAGE_NULL_COUNT).all()
    slots = batch.pages["num_values"].astype(np.int64)
    vals = slots - batch.pages["num_nulls"]
    ref = pqref.decode_batch(batch)
    assert np.array_equal(vals, ref.page_value_counts.astype(np.int64))


@pytest.mark.gpu
def test_right_counts_start_values_beside_levels(decoder):
    """Correct header counts: no re-run, and the plan launches one kernel fewer than level-first (no offset
    scan: the host has the offsets)."""
    batch = writer.build_batch(_c3_like())
    plan = _plan_run(decoder, batch)
    assert plan.null_hint_fallbacks == 0
    decoder.set_dispatch(abi.DISPATCH_NULL_HINTS, 0)
    try:
        plan0 = _plan_run(decoder, batch, launches=1)
    finally:
        decoder.set_dispatch(abi.DISPATCH_NULL_HINTS, 1)
    assert plan0.kernel_count == plan.kernel_count + 1
    plan.close()
    plan0.close()


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["plus1", "minus1", "zero", "all", "last_page", "every_page"])
def test_wrong_header_counts_rerun_level_first(decoder, how):
    """A header num_nulls that disagrees with the levels: the launch is re-run level-first (one fallback,
    kept for the next launch), and values / offsets / levels equal the oracle's."""
    chunks = _c3_like()
    for ch in chunks:
        pages = ch.pages if how == "every_page" else [ch.pages[-1 if how == "last_page" else 1]]
        for pg in pages:
            if how in ("plus1", "last_page", "every_page"):
                pg.num_nulls = min(pg.num_nulls + 1, pg.num_values)
            elif how == "minus1":
                pg.num_nulls = max(pg.num_nulls - 1, 0)
            elif how == "zero":
                pg.num_nulls = 0
            else:
                pg.num_nulls = pg.num_values
    batch = writer.build_batch(chunks)
    plan = _plan_run(decoder, batch)
    assert plan.null_hint_fallbacks == 1
    plan.close()


@pytest.mark.gpu
def test_wrong_header_count_one_column_of_many(decoder):
    """Only one page of one column is wrong: the whole plan re-runs level-first; through pqg_decode too."""
    chunks = _c3_like(seed=9)
    chunks[3].pages[2].num_nulls += 3
    run_both(decoder, chunks)


@pytest.mark.gpu
def test_wrong_header_count_with_page_counts(decoder):
    """pqg_decode's per-page value counts (copied after the first launch) are refreshed by the re-run."""
    chunks = _c3_like(seed=5, page_rows=3000)
    chunks[0].pages[0].num_nulls = 0
    batch = writer.build_batch(chunks)
    ref = pqref.decode_batch(batch)
    counts = torch.zeros(batch.n_pages, dtype=torch.int32, device=decoder.device)
    cols, st = decoder.decode(decoder.upload(batch), page_counts=counts)
    assert st.code == 0
    assert np.array_equal(counts.cpu().numpy().view(np.uint32), ref.page_value_counts)
    _check(batch, ref, cols)


@pytest.mark.gpu
def test_header_count_past_the_slots_is_not_used(decoder):
    """num_nulls > num_values: not a usable hint (the plan stays level-first), same results."""
    chunks = _c3_like(seed=7)
    chunks[1].pages[0].num_nulls = chunks[1].pages[0].num_values + 5
    batch = writer.build_batch(chunks)
    plan = _plan_run(decoder, batch, launches=1)
    assert plan.null_hint_fallbacks == 0
    plan.close()


@pytest.mark.gpu
def test_v1_and_v2_pages_mixed(decoder):
    """A nullable column with a V1 page: no hints for the plan (level-first), same results."""
    a = _c3_like(seed=11, version=2)
    b = _c3_like(seed=11, version=1)
    a[2].pages[1] = b[2].pages[1]
    run_both(decoder, a)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(6))
def test_level_errors_with_header_counts(decoder, seed):
    """Corrupted V2 level sections under right header counts: the first error (code, page, slot) is the
    oracle's (the hinted launch is re-run level-first, whose error order is the reference's)."""
    rng = np.random.default_rng(100 + seed)
    chunks = _c3_like(seed=seed, page_rows=2000)
    for ch in chunks:
        for pg in ch.pages:
            if rng.random() < 0.3:
                body = bytearray(pg.body)
                hi = pg.rl_byte_length + pg.dl_byte_length
                if hi:
                    body[rng.integers(0, hi)] = int(rng.integers(0, 256))
                pg.body = bytes(body)
    batch = writer.build_batch(chunks)
    ref = pqref.decode_batch(batch)
    run_both(decoder, chunks, expect_error=ref.code != 0)


@pytest.mark.gpu
def test_value_error_with_right_header_counts(decoder):
    """A value-section error (truncated PLAIN data) on a page whose header count is right: reported from
    the hinted launch itself, equal to the oracle's."""
    chunks = _c3_like(seed=13, page_rows=4000)
    pg = chunks[2].pages[3]
    pg.body = pg.body[:-20]
    run_both(decoder, chunks, expect_error=True)
