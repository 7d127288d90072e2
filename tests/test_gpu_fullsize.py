"""BASELINE configs at full size on the GPU: C2 (100M int64 RLE_DICTIONARY, 5,000
pages, Zipf 1.5 and 2.0), C3 (8 optional columns x 100M slots), C5 (100M LIST<int64> records).

At these sizes the oracle would take minutes, so parity is checked through size-independent
properties: the decoded columns equal the values the writer was given (bit patterns; BYTE_ARRAY
offsets and bytes), the levels equal the generated levels, and the assembled list offsets /
validity equal the generated list structure. A sample of pages is also decoded by the oracle
(oracle/pqref.c) and compared with the same expected values.

The C2 cases check the FIRST launch of a freshly created plan (the fused kernel's walk -> expansion
hand-off across 5,000 pages on every XCD: a stale run record would show here, not after warm-up
launches have rewritten the same records) and again after more launches of the same plan.
"""
import os
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

import workloads as WL  # noqa: E402
from pqgpu import abi  # noqa: E402
from tools.synth import writer  # noqa: E402

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

FULL = 100_000_000


def oracle_sample(work, n_pages=20):
    """The oracle decodes the first n_pages of every column; its values equal the expected prefix."""
    from oracle import pqref
    for ch, ex in zip(work.chunks, work.expect):
        c = writer.ColumnChunk(**{k: getattr(ch, k) for k in ("physical_type", "max_rep", "max_def", "type_length",
                                                               "dict_page", "dict_num_values", "dict_encoding")})
        c.pages = ch.pages[:n_pages]
        r = pqref.decode_batch(writer.build_batch([c]))
        assert r.code == 0, r.status
        got = r.columns[0]
        n = got["n_values"]
        if isinstance(ex.values, writer.BinaryValues):
            assert list(got["values"]) == [ex.values[k] for k in range(n)]
        else:
            assert np.array_equal(np.asarray(got["values"]).view(np.uint8),
                                  np.ascontiguousarray(ex.values[:n]).view(np.uint8))


@pytest.mark.parametrize("a", [1.5, 2.0])
def test_c2_fresh_plan_first_launch(decoder, a):
    work = WL.c2(FULL, a=a)
    batch = writer.build_batch(work.chunks)
    assert batch.n_pages == 5000
    oracle_sample(work)
    dbatch = decoder.upload(batch)
    cols = decoder.alloc_columns(batch)        # poisoned (0xA5) outputs
    plan = decoder.plan(dbatch, cols)
    plan.launch()                              # first launch of a fresh plan
    rc, st = plan.sync()
    assert rc == 0, st.message
    WL.verify(cols, work, "first launch")
    for _ in range(5):
        plan.launch()
    rc, st = plan.sync()
    assert rc == 0, st.message
    WL.verify(cols, work, "after 6 launches")
    plan.close()


def test_c2_many_fresh_plans(decoder):
    """Ten freshly created plans over the same 5,000 pages, each checked after its first launch
    (scratch and flags are new memory every time)."""
    work = WL.c2(FULL)
    batch = writer.build_batch(work.chunks)
    dbatch = decoder.upload(batch)
    exp = torch.from_numpy(work.expect[0].values).to(decoder.device)
    for k in range(10):
        cols = decoder.alloc_columns(batch)
        plan = decoder.plan(dbatch, cols)
        plan.launch()
        rc, st = plan.sync()
        assert rc == 0, st.message
        assert torch.equal(cols[0].typed(), exp), f"plan {k}: first launch differs"
        plan.close()


def test_c3_full(decoder):
    work = WL.c3_mixed(FULL, log=False)
    oracle_sample(work, 10)
    batch = writer.build_batch(work.chunks)
    dbatch = decoder.upload(batch)
    cols, st = decoder.decode(dbatch)          # sizes the BYTE_ARRAY buffers
    WL.verify(cols, work, "decode")
    plan = decoder.plan(dbatch, cols)
    for _ in range(3):
        plan.launch()
    rc, st = plan.sync()
    assert rc == 0, st.message
    WL.verify(cols, work, "plan")
    plan.close()


def test_c5_full_with_assembly(decoder):
    work = WL.c5_levels(FULL)
    oracle_sample(work)
    batch = writer.build_batch(work.chunks)
    dbatch = decoder.upload(batch)
    cols, st = decoder.decode(dbatch)
    WL.verify(cols, work, "decode")
    n_slots = batch.column_slots[0]
    got = decoder.assemble([abi.OPTIONAL, abi.REPEATED, abi.OPTIONAL], n_slots, cols[0].def_levels, cols[0].rep_levels)
    lens, null_list = work.lists["lens"], work.lists["null_list"]
    assert got["records"] == lens.size
    dev = decoder.device
    v0 = got["nodes"][0]["validity"]
    assert torch.equal(v0, torch.from_numpy((~null_list).astype(np.uint8)).to(dev)), "list validity"
    offs = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)).to(dev)
    assert torch.equal(got["nodes"][1]["offsets"], offs), "list offsets"
    dl = work.expect[0].def_levels
    elem_valid = (dl[dl >= 2] == 3).astype(np.uint8)
    assert torch.equal(got["nodes"][2]["validity"], torch.from_numpy(elem_valid).to(dev)), "element validity"


def test_c4_lineitem_row_groups(decoder):
    """C4: four 1M-row lineitem row groups (64 column chunks: DELTA keys / dates, PLAIN doubles,
    dictionary int32 + strings, PLAIN comments) in one batch, each chunk == its generated values;
    an oracle sample of every column first."""
    import lineitem as LI
    work = LI.make_c4(4_000_000)
    oracle_sample(WL.Workload("c4 rg0", work.chunks[:16], work.expect[:16]), 5)
    batch = writer.build_batch(work.chunks)
    dbatch = decoder.upload(batch)
    cols, st = decoder.decode(dbatch)
    WL.verify(cols, work, "decode")
    plan = decoder.plan(dbatch, cols)
    plan.launch()
    rc, st = plan.sync()
    assert rc == 0, st.message
    WL.verify(cols, work, "plan")
    plan.close()


def poison(cols, byte=0xA5):
    for c in cols:
        for t in (c.values, c.def_levels, c.rep_levels, c.binary_data):
            if t is not None:
                t.fill_(byte)


def test_c4_configured_shard(decoder):
    """C4 at its configured per-GPU size: 1 B rows / 8 GPUs = 125 M rows = 125 row groups of 1 M rows,
    100,000 pages, 636 pqg columns (BASELINE configs[3]; the row-group split of
    ParquetInputFormat.java:350,786 as pqgpu.dist.shard_row_groups makes it for rank 0 of 8 with the
    1 B-row table). An oracle sample of every column first; then the FIRST launch of a fresh plan
    into poisoned outputs must give every row group x column slice == its generated values, and
    again after more launches."""
    import lineitem as LI
    shard = LI.Shard(1_000_000_000, world=8, rank=0)
    assert len(shard.mine) == 125 and shard.batch.n_pages == 100_000
    oracle_sample(WL.Workload("c4 rg0", shard.templates[0][0], shard.templates[0][1]), 5)
    dbatch = decoder.upload(shard.batch)
    cols, st = decoder.decode(dbatch)          # sizes the BYTE_ARRAY buffers
    poison(cols)
    plan = decoder.plan(dbatch, cols)
    plan.launch()                              # first launch of a fresh plan
    rc, st = plan.sync()
    assert rc == 0, st.message
    shard.verify(cols, decoder.device, "first launch")
    for _ in range(3):
        plan.launch()
    rc, st = plan.sync()
    assert rc == 0, st.message
    shard.verify(cols, decoder.device, "after 4 launches")
    plan.close()
