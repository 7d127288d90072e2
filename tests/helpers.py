"""Shared test-input builders (synthetic columns in the shapes of BASELINE.json's configs)."""
import numpy as np

from pqgpu import abi
from tools.synth import writer


def zipf_dict_column(n, card=1000, a=1.5, seed=0, physical_type=abi.INT64, max_run=4096):
    rng = np.random.default_rng(seed)
    if physical_type in (abi.INT64,):
        dvals = rng.integers(-2**63, 2**63 - 1, size=card, dtype=np.int64)
    elif physical_type == abi.INT32:
        dvals = rng.integers(-2**31, 2**31 - 1, size=card, dtype=np.int64).astype(np.int32)
    elif physical_type == abi.DOUBLE:
        dvals = rng.standard_normal(card)
    else:
        dvals = rng.standard_normal(card).astype(np.float32)
    runs = np.minimum(rng.zipf(a, size=n // 2 + 16), max_run)
    ids = np.repeat(rng.integers(0, card, size=runs.size), runs)[:n]
    return dvals[ids]


def nulls(n_slots, frac, seed):
    rng = np.random.default_rng(seed)
    return (rng.random(n_slots) >= frac).astype(np.uint8)


def make(physical_type, values, encoding, **kw):
    return writer.write_column_chunk(physical_type, values, encoding, **kw)


def assert_same(gpu_res, ref_col, physical_type):
    if physical_type == abi.BYTE_ARRAY:
        g, r = list(gpu_res), list(ref_col)
        assert len(g) == len(r), (len(g), len(r))
        bad = [i for i in range(len(g)) if g[i] != r[i]]
        assert not bad, f"{len(bad)} mismatches, first at {bad[:5]}: gpu={[g[i] for i in bad[:3]]} ref={[r[i] for i in bad[:3]]}"
        return
    g = np.asarray(gpu_res)
    r = np.asarray(ref_col)
    assert g.shape == r.shape, (g.shape, r.shape)
    if g.dtype.kind == "f":
        g = g.view(np.uint32 if g.dtype.itemsize == 4 else np.uint64)
        r = r.view(g.dtype)
    if g.dtype.kind == "V":
        g = g.view(np.uint8)
        r = r.view(np.uint8)
    bad = np.nonzero(g != r)[0]
    assert bad.size == 0, f"{bad.size} mismatches, first at {bad[:5]}: gpu={g[bad[:5]]} ref={r[bad[:5]]}"
