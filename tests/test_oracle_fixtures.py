"""Pin the oracle to real files: the reference's own fixture files (parquet-mr 1.9 / 1.13
and Arrow-written, under parquet-hadoop/src/test/resources and parquet-avro/src/test/resources)
and pyarrow-written files with the hot-path encodings. Expected values were read by
pyarrow (tests/golden/make_golden.py)."""
import numpy as np
import pytest

from oracle import pqref
from pqgpu import abi

from fixtures import batch_of, chunk_cases, load_chunk

CASES = list(chunk_cases())


@pytest.mark.parametrize("name,c", CASES, ids=[f"{n}:{c['key']}:{c['path']}" for n, c in CASES])
def test_oracle_decodes_fixture(name, c):
    ch, expected = load_chunk(name, c)
    assert sum(p.num_values for p in ch.pages) == c["num_values"]
    res = pqref.decode_batch(batch_of(ch))
    assert res.code == 0, res.status
    got = res.columns[0]["values"]
    if ch.physical_type == abi.BYTE_ARRAY:
        assert got == expected
    else:
        g = np.asarray(got)
        e = np.asarray(expected)
        assert g.shape == e.shape
        if g.dtype.kind == "f":
            g, e = g.view(np.uint8), e.view(np.uint8)
        assert np.array_equal(g, e)
    # levels: every slot decoded, non-null count agrees
    if c["max_def"] > 0:
        dl = res.columns[0]["def_levels"]
        assert dl.size == c["num_values"]
        assert int((dl == c["max_def"]).sum()) == len(expected)


def test_fixture_set_covers_hot_path():
    encs = set()
    for _, c in CASES:
        encs.update(c["encodings"])
    assert {"PLAIN", "PLAIN_DICTIONARY", "RLE_DICTIONARY", "DELTA_BINARY_PACKED", "RLE", "BIT_PACKED"} <= encs
    creators = {c["created_by"].split(" ")[0] for _, c in CASES}
    assert "parquet-mr" in creators
