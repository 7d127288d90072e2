"""Synthetic inputs of the BASELINE.json configs, with the values that were written.

One place generates every workload that bench.py, tools/bench_suite.py and the full-size GPU tests
(tests/test_gpu_fullsize.py) use, so the timed inputs are exactly the verified ones. Each generator
returns a `Workload`: the parquet-mr-identical column chunks (pqgpu.writer) plus, per column, what
the reference reader hands back for them — the dense non-null values in slot order and the per-slot
def / rep levels (ColumnReaderBase.readPageV1/V2 + the value reader, SURVEY.md §3 call stack A).

Workloads:
  c2 / c2_zipf2  C2: 100M int64 RLE_DICTIONARY, 1k-card dictionary (w = 10), Zipf(1.5 / 2.0) runs
  c3_mixed       C3: 8 optional columns (2 int32 + 2 int64 DELTA_BINARY_PACKED, 2 double PLAIN,
                 2 BYTE_ARRAY PLAIN 4-32 B), 10 % nulls, RLE def levels, V2 pages
  c5_levels      C5: LIST<int64> (Poisson(3) lengths, 10 % null lists / elements), rep + def levels
  c4_lineitem    C4: TPC-H lineitem-shaped 16 columns (see make_c4)
"""
import os
import sys
from dataclasses import dataclass, field
from typing import List

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (os.path.join(REPO, "parquet-mr_amd"), REPO):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from pqgpu import abi  # noqa: E402
from tools.synth import writer  # noqa: E402


@dataclass
class Expected:
    values: object                 # numpy array, or writer.BinaryValues for BYTE_ARRAY
    def_levels: np.ndarray = None  # u8 per slot (None: required)
    rep_levels: np.ndarray = None


@dataclass
class Workload:
    name: str
    chunks: List[writer.ColumnChunk]
    expect: List[Expected] = field(default_factory=list)
    note: str = ""


def nulls(n, frac, seed):
    return (np.random.default_rng(seed).random(n) >= frac).astype(np.uint8)


def make_c2(n_rows, seed_dict=42, seed_runs=43, a=1.5, card=1000, max_run=4096, page_rows=20000):
    """C2: the dictionary column as parquet-mr writes it (ids in first-appearance order, 1-byte bit
    width + RLE/bit-packed hybrid ids, PLAIN dictionary page, V1 pages of 20,000 values)."""
    rng_d = np.random.default_rng(seed_dict)
    dict_vals = rng_d.integers(-2**63, 2**63 - 1, size=card, dtype=np.int64, endpoint=True)
    rng = np.random.default_rng(seed_runs)
    runs = []
    total = 0
    while total < n_rows:
        r = np.minimum(rng.zipf(a, size=1 << 20), max_run)
        runs.append(r)
        total += int(r.sum())
    runs = np.concatenate(runs)
    run_ids = rng.integers(0, card, size=runs.size)
    cut = np.searchsorted(np.cumsum(runs), n_rows)
    runs, run_ids = runs[:cut + 1], run_ids[:cut + 1]
    ids = np.repeat(run_ids, runs)[:n_rows]
    ids_fa, order = writer.first_appearance_ids(ids)
    chunk = writer.write_dict_column_from_ids(abi.INT64, dict_vals[order], ids_fa, page_rows=page_rows)
    return chunk, dict_vals, ids


def binary_take(words, ids):
    """BinaryValues of words[ids] (words: list of bytes; vectorized)."""
    lens = np.array([len(w) for w in words], dtype=np.int64)
    starts = np.concatenate([[0], np.cumsum(lens)])[:-1]
    blob = np.frombuffer(b"".join(words), dtype=np.uint8)
    vl = lens[ids]
    offs = np.concatenate([[0], np.cumsum(vl)]).astype(np.int64)
    pos = np.arange(int(offs[-1]), dtype=np.int64) - np.repeat(offs[:-1], vl) + np.repeat(starts[ids], vl)
    return writer.BinaryValues(offs, blob[pos])


def c2(rows, a=1.5, seed_runs=43):
    ch, dv, ids = make_c2(rows, a=a, seed_runs=seed_runs)
    return Workload(f"c2 zipf={a}", [ch], [Expected(dv[ids])])


def c3_mixed(rows, log=True):
    rng = np.random.default_rng(7)
    dl = nulls(rows, 0.1, 8)
    n = int(dl.sum())
    out, exp = [], []
    for k in range(2):
        walk = np.cumsum(rng.integers(-100, 1000, size=n)).astype(np.int64)
        v32 = (walk % (1 << 30)).astype(np.int32)
        v64 = walk * 1000 + k
        vd = rng.standard_normal(n)
        vb = writer.BinaryValues.random(n, 4, 32, seed=k)
        out.append(writer.write_column_chunk(abi.INT32, v32, abi.DELTA_BINARY_PACKED, def_levels=dl, max_def=1, version=2))
        out.append(writer.write_column_chunk(abi.INT64, v64, abi.DELTA_BINARY_PACKED, def_levels=dl, max_def=1, version=2))
        out.append(writer.write_column_chunk(abi.DOUBLE, vd, abi.PLAIN, def_levels=dl, max_def=1, version=2))
        out.append(writer.write_column_chunk(abi.BYTE_ARRAY, vb, abi.PLAIN, def_levels=dl, max_def=1, version=2))
        exp += [Expected(v32, dl), Expected(v64, dl), Expected(vd, dl), Expected(vb, dl)]
        if log:
            print(f"[gen c3_mixed] {len(out)} of 8 columns", file=sys.stderr, flush=True)
    return Workload("c3_mixed", out, exp)


C3_PARTS = {"c3_delta": (0, 1, 4, 5), "c3_double": (2, 6), "c3_strings": (3, 7)}


def c5_levels(recs):
    rng = np.random.default_rng(7)
    lens = rng.poisson(3, size=recs)
    null_list = rng.random(recs) < 0.1
    slots = np.where(null_list | (lens == 0), 1, lens)
    n_slots = int(slots.sum())
    starts = np.concatenate([[0], np.cumsum(slots)[:-1]])
    rl = np.ones(n_slots, dtype=np.uint8)
    rl[starts] = 0
    dl = np.full(n_slots, 3, dtype=np.uint8)
    dl[rng.random(n_slots) < 0.1] = 2
    dl[starts[null_list]] = 0
    dl[starts[~null_list & (lens == 0)]] = 1
    n = int((dl == 3).sum())
    vals = rng.integers(-2**40, 2**40, size=n)
    ch = writer.write_column_chunk(abi.INT64, vals, abi.PLAIN, def_levels=dl, rep_levels=rl, max_def=3, max_rep=1,
                                   page_rows=20000)
    w = Workload("c5_levels", [ch], [Expected(vals, dl, rl)])
    # list structure the assembly must reproduce: per record, null list / element count
    w.lists = {"null_list": null_list, "lens": np.where(null_list, 0, lens)}
    return w


def verify(cols, work, what=""):
    """Decoded device columns == the written values (bit patterns; BYTE_ARRAY: offsets and bytes)
    and levels. Compared on the device (full-size columns: no host round trip). Raises
    AssertionError naming the first mismatching column."""
    import torch
    assert len(cols) == len(work.expect), (len(cols), len(work.expect))
    for i, (col, ex) in enumerate(zip(cols, work.expect)):
        dev = col.values.device
        tag = f"{what} {work.name} column {i}"
        if isinstance(ex.values, writer.BinaryValues):
            n = len(ex.values)
            assert col.n_values == n, (tag, col.n_values, n)
            offs = torch.from_numpy(np.asarray(ex.values.offsets, dtype=np.int64)).to(dev)
            assert torch.equal(col.offsets(), offs), f"{tag}: offsets differ"
            total = int(ex.values.offsets[-1])
            got = col.binary_data[:total]
            assert torch.equal(got, torch.from_numpy(np.asarray(ex.values.data[:total], dtype=np.uint8)).to(dev)), \
                f"{tag}: value bytes differ"
        else:
            v = np.ascontiguousarray(ex.values)
            assert col.n_values == v.size, (tag, col.n_values, v.size)
            got = col.values[: v.nbytes]
            assert torch.equal(got, torch.from_numpy(v.view(np.uint8)).to(dev)), f"{tag}: values differ"
        for name, lv in (("def", ex.def_levels), ("rep", ex.rep_levels)):
            if lv is None:
                continue
            t = col.def_levels if name == "def" else col.rep_levels
            assert torch.equal(t[: lv.size], torch.from_numpy(np.ascontiguousarray(lv, dtype=np.uint8)).to(dev)), \
                f"{tag}: {name} levels differ"


def generate(name, rows):
    if name == "c2":
        return c2(rows)
    if name == "c2_zipf2":
        return c2(rows, a=2.0)
    if name == "c3_mixed":
        return c3_mixed(rows)
    if name in C3_PARTS:  # C3's columns of one kind alone (kernel times without the other columns' overlap)
        w = c3_mixed(rows)
        keep = C3_PARTS[name]
        return Workload(name, [w.chunks[i] for i in keep], [w.expect[i] for i in keep])
    if name == "c5_levels":
        return c5_levels(rows)
    if name == "c4_lineitem":
        from lineitem import make_c4
        return make_c4(rows)
    raise ValueError(name)
