"""GPU record assembly (pqg_assemble) vs the oracle restatement of parquet-mr's Dremel automaton
(RecordReaderImplementation.read, oracle/assembly.py pinned to TestColumnIO.expectedEventsForR1):
offsets of every REPEATED node and validity of every OPTIONAL node, bit-exact."""
import numpy as np
import pytest
import torch

from oracle import assembly as A
from oracle import pqref
from pqgpu import abi
from tools.synth import writer

from test_oracle_assembly import PAPER, stripes

pytestmark = pytest.mark.gpu


def gpu_vs_oracle(decoder, path, rl, dl, vals=None):
    names = [f"n{k}" for k in range(len(path))]
    n = len(dl)
    lv = A.levels_of(path)
    if vals is None:
        vals = [0] * int(sum(1 for d in dl if d >= lv[-1][1]))
    exp = A.columnar(path, A.fsm_events(path, names, rl, dl, vals))
    dev = decoder.device
    dt = torch.tensor(np.asarray(dl, dtype=np.uint8), device=dev) if lv[-1][1] > 0 else None
    rt = torch.tensor(np.asarray(rl, dtype=np.uint8), device=dev) if lv[-1][0] > 0 else None
    got = decoder.assemble(path, n, dt, rt)
    assert got["records"] == exp["records"]
    for k, rp in enumerate(path):
        node = got["nodes"][k]
        if rp == abi.OPTIONAL:
            assert node["validity"].cpu().numpy().tolist() == exp["validity"][k], f"validity of node {k}"
        if rp == abi.REPEATED:
            assert node["offsets"].cpu().numpy().tolist() == exp["offsets"][k], f"offsets of node {k}"
    return got, exp


@pytest.mark.parametrize("leaf", list(PAPER))
def test_paper_records(decoder, leaf):
    names, path, r1, r2 = PAPER[leaf]
    rl, dl, vals = stripes(r1 + r2)
    gpu_vs_oracle(decoder, path, rl, dl, vals)


def random_levels(path, n, rng):
    """A valid level sequence for `path` (as a writer produces): r_0 = 0; slot i may continue
    repeated node r only if slot i - 1 reached it (d_{i-1} >= DR[r]), and then has it defined
    (d_i >= DR[r]). (On sequences no writer produces the automaton's output is not specified.)"""
    lv = A.levels_of(path)
    max_r, max_d = lv[-1]
    DR = [0] + [lv[k][1] for k in range(len(path)) if path[k] == A.REPEATED]
    rl = np.zeros(n, dtype=np.uint8)
    dl = np.zeros(n, dtype=np.uint8)
    u = rng.random((n, 2))
    prev_d = 0
    for i in range(n):
        reach = max(q for q in range(max_r + 1) if DR[q] <= prev_d) if i else 0
        r = int(u[i, 0] * (reach + 1))
        d = DR[r] + int(u[i, 1] * (max_d - DR[r] + 1))
        rl[i], dl[i] = r, min(d, max_d)
        prev_d = dl[i]
    return rl, dl


PATHS = [
    [A.OPTIONAL, A.REPEATED, A.OPTIONAL],            # Arrow LIST<optional> (config 5)
    [A.REPEATED],                                    # repeated primitive
    [A.REQUIRED],
    [A.OPTIONAL],
    [A.OPTIONAL, A.OPTIONAL, A.OPTIONAL],
    [A.REPEATED, A.REPEATED, A.OPTIONAL],            # Name.Language.Country
    [A.OPTIONAL, A.REPEATED, A.REQUIRED, A.REPEATED, A.OPTIONAL],
    [A.REPEATED, A.OPTIONAL, A.REPEATED, A.OPTIONAL, A.REPEATED, A.REQUIRED],
    [A.REQUIRED, A.REPEATED, A.REQUIRED, A.REQUIRED, A.OPTIONAL],
]


@pytest.mark.parametrize("pi", range(len(PATHS)))
@pytest.mark.parametrize("n", [1, 777, 20000])
def test_random_levels(decoder, pi, n):
    rng = np.random.default_rng(pi * 100 + n)
    rl, dl = random_levels(PATHS[pi], n, rng)
    gpu_vs_oracle(decoder, PATHS[pi], rl.tolist(), dl.tolist())


def test_empty_column(decoder):
    got = decoder.assemble([A.OPTIONAL, A.REPEATED, A.OPTIONAL], 0, torch.zeros(1, dtype=torch.uint8, device="cuda"),
                           torch.zeros(1, dtype=torch.uint8, device="cuda"))
    assert got["records"] == 0 and got["nodes"][1]["offsets"].cpu().tolist() == [0]


def test_decode_then_assemble_config5(decoder):
    """Config 5 shape end to end: the page levels decoded by pqg_decode feed pqg_assemble."""
    rng = np.random.default_rng(11)
    recs = 30_000
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
    vals = rng.integers(-2**40, 2**40, size=int((dl == 3).sum())).astype(np.int64)
    ch = writer.write_column_chunk(abi.INT64, vals, abi.PLAIN, def_levels=dl, rep_levels=rl, max_def=3, max_rep=1,
                                   page_rows=5000, version=2)
    batch = writer.build_batch([ch])
    cols, st = decoder.decode(decoder.upload(batch))
    n = batch.column_slots[0]
    got, exp = gpu_vs_oracle(decoder, [A.OPTIONAL, A.REPEATED, A.OPTIONAL], rl.tolist(), dl.tolist(), vals.tolist())
    got2 = decoder.assemble([A.OPTIONAL, A.REPEATED, A.OPTIONAL], n, cols[0].def_levels, cols[0].rep_levels)
    assert got2["records"] == recs
    for k in range(3):
        for key in ("validity", "offsets"):
            a, b = got["nodes"][k][key], got2["nodes"][k][key]
            assert (a is None) == (b is None) and (a is None or torch.equal(a, b))
    assert np.array_equal(cols[0].numpy(), vals)
