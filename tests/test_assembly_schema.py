"""Record assembly over every leaf of a schema: the oracle restates RecordReaderImplementation's
automaton across leaves (oracle/assembly.py fsm_events_multi, pinned to the FULL
TestColumnIO.expectedEventsForR1 interleaving, parquet-column/src/test/java/org/apache/parquet/io/TestColumnIO.java:114-142);
the shredder in tests/records.py is pinned to TestColumnIO.testWriteWithGroupWriter's stripes (:596-620).
The `gpu` tests compare pqg_assemble_schema with the oracle's columnar form on random nested records."""
import numpy as np
import pytest

from oracle import assembly as A

from records import flat_schema, random_record, rebuild, shred
from test_oracle_assembly import EXPECTED_EVENTS_R1, PAPER, stripes

R, O, P = A.REQUIRED, A.OPTIONAL, A.REPEATED
N = A.Node

# org.apache.parquet.example.Paper.schema
DOCUMENT = [N("DocId", R), N("Links", O, [N("Backward", P), N("Forward", P)]),
            N("Name", P, [N("Language", P, [N("Code", R), N("Country", O)]), N("Url", O)])]
LEAVES = ["DocId", "Links.Backward", "Links.Forward", "Name.Language.Code", "Name.Language.Country", "Name.Url"]
R1 = {"DocId": 10, "Links": {"Forward": [20, 40, 60]},
      "Name": [{"Language": [{"Code": b"en-us", "Country": b"us"}, {"Code": b"en"}], "Url": b"http://A"},
               {"Url": b"http://B"}, {"Language": [{"Code": b"en-gb", "Country": b"gb"}]}]}
R2 = {"DocId": 20, "Links": {"Backward": [10, 30], "Forward": [80]}, "Name": [{"Url": b"http://C"}]}

# a second schema: optional and repeated groups at several depths, required leaves under repeated
SCHEMA_B = [N("a", O, [N("b", P, [N("c", O), N("d", R)]), N("e", O)]),
            N("f", P, [N("g", P, [N("h", P)]), N("i", R)]),
            N("j", R)]


def test_multi_leaf_automaton_reproduces_expected_events_for_r1():
    cols = [stripes(PAPER[k][2]) for k in LEAVES]
    ev = A.fsm_events_multi(DOCUMENT, cols)
    assert A.event_strings_multi(ev) == EXPECTED_EVENTS_R1


def test_shredder_matches_the_reference_writer():
    """testWriteWithGroupWriter: the stripes of r1 and r2 per leaf."""
    got = shred(DOCUMENT, [R1, R2])
    for k, (rl, dl, vals) in zip(LEAVES, got):
        erl, edl, evals = stripes(PAPER[k][2] + PAPER[k][3])
        assert rl.tolist() == erl and dl.tolist() == edl and vals == evals, k


@pytest.mark.parametrize("roots", [DOCUMENT, SCHEMA_B], ids=["document", "schema_b"])
def test_automaton_rebuilds_random_records(roots):
    rng = np.random.default_rng(len(roots))
    recs = [random_record(roots, rng) for _ in range(300)]
    ev = A.fsm_events_multi(roots, shred(roots, recs))
    assert rebuild(roots, ev) == recs


def test_multi_columnar_equals_per_leaf_columnar():
    rng = np.random.default_rng(5)
    recs = [random_record(SCHEMA_B, rng) for _ in range(200)]
    cols = shred(SCHEMA_B, recs)
    multi = A.columnar_multi(SCHEMA_B, A.fsm_events_multi(SCHEMA_B, cols))
    for chain, (rl, dl, vals) in zip(A.schema_leaves(SCHEMA_B), cols):
        path = [n.repetition for n in chain]
        names = [n.name for n in chain]
        one = A.columnar(path, A.fsm_events(path, names, rl, dl, vals))
        assert one["records"] == multi["records"]
        for k, v in one["validity"].items():
            assert multi["validity"][".".join(names[:k + 1])] == v
        for k, v in one["offsets"].items():
            assert multi["offsets"][".".join(names[:k + 1])] == v


def gpu_schema_vs_oracle(decoder, roots, recs):
    import torch
    cols = shred(roots, recs)
    exp = A.columnar_multi(roots, A.fsm_events_multi(roots, cols))
    nodes, leaf_idx, names = flat_schema(roots)
    leaves = []
    for chain, k, (rl, dl, _) in zip(A.schema_leaves(roots), leaf_idx, cols):
        max_r, max_d = A.levels_of([n.repetition for n in chain])[-1]
        dt = torch.tensor(dl, device=decoder.device) if max_d > 0 else None
        rt = torch.tensor(rl, device=decoder.device) if max_r > 0 else None
        leaves.append((k, dt, rt, len(dl)))
    got = decoder.assemble_schema(nodes, leaves)
    assert got["records"] == exp["records"] == len(recs)
    for k, (parent, rp) in enumerate(nodes):
        if rp == A.OPTIONAL:
            assert got["nodes"][k]["validity"].cpu().numpy().tolist() == exp["validity"][names[k]], names[k]
        if rp == A.REPEATED:
            assert got["nodes"][k]["offsets"].cpu().numpy().tolist() == exp["offsets"][names[k]], names[k]


@pytest.mark.gpu
def test_gpu_paper_records(decoder):
    gpu_schema_vs_oracle(decoder, DOCUMENT, [R1, R2])


@pytest.mark.gpu
@pytest.mark.parametrize("roots,n", [(DOCUMENT, 3000), (SCHEMA_B, 3000), (SCHEMA_B, 20000)],
                         ids=["document", "schema_b", "schema_b_large"])
def test_gpu_random_records(decoder, roots, n):
    rng = np.random.default_rng(n + len(roots))
    gpu_schema_vs_oracle(decoder, roots, [random_record(roots, rng) for _ in range(n)])


@pytest.mark.gpu
def test_gpu_leaves_that_disagree(decoder):
    """Two leaves under one repeated group with different element counts: PQG_ERR_CORRUPT."""
    import torch
    from pqgpu import abi, native
    roots = [N("g", P, [N("x", R), N("y", R)])]
    nodes, leaf_idx, _ = flat_schema(roots)
    rl1 = torch.tensor([0, 1, 1], dtype=torch.uint8, device=decoder.device)
    dl1 = torch.tensor([1, 1, 1], dtype=torch.uint8, device=decoder.device)
    rl2 = torch.tensor([0, 1], dtype=torch.uint8, device=decoder.device)
    dl2 = torch.tensor([1, 1], dtype=torch.uint8, device=decoder.device)
    with pytest.raises(native.PqgError) as e:
        decoder.assemble_schema(nodes, [(leaf_idx[0], dl1, rl1, 3), (leaf_idx[1], dl2, rl2, 2)])
    assert e.value.code == abi.ERR_CORRUPT
