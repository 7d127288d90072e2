"""GPU decode of every golden fixture column chunk (reference parquet-mr/Arrow files and
pyarrow-written encodings) vs the expected values and the oracle."""
import numpy as np
import pytest

from oracle import pqref
from pqgpu import abi

from fixtures import batch_of, chunk_cases, load_chunk
from helpers import assert_same

pytestmark = pytest.mark.gpu
CASES = list(chunk_cases())
GPU_DBA = True  # DELTA_BYTE_ARRAY on the device


@pytest.mark.parametrize("name,c", CASES, ids=[f"{n}:{c['key']}:{c['path']}" for n, c in CASES])
def test_gpu_decodes_fixture(decoder, name, c):
    ch, expected = load_chunk(name, c)
    batch = batch_of(ch)
    cols, st = decoder.decode(decoder.upload(batch), check=False)
    if "DELTA_BYTE_ARRAY" in c["encodings"] and not GPU_DBA:
        # DELTA_BYTE_ARRAY is the next row: reported, not silently wrong
        assert st.code == abi.ERR_UNSUPPORTED
        return
    assert st.code == 0, st.message
    got = cols[0].numpy()
    assert_same(got, expected, ch.physical_type)
    ref = pqref.decode_batch(batch)
    if c["max_def"] > 0:
        assert np.array_equal(cols[0].def_levels[:batch.column_slots[0]].cpu().numpy(), ref.columns[0]["def_levels"])
    if c["max_rep"] > 0:
        assert np.array_equal(cols[0].rep_levels[:batch.column_slots[0]].cpu().numpy(), ref.columns[0]["rep_levels"])


def test_gpu_all_fixtures_one_batch(decoder):
    """Every fixture chunk decoded in ONE pqg_decode call (many columns, mixed encodings)."""
    chunks, exp = [], []
    for name, c in CASES:
        ch, e = load_chunk(name, c)
        if "DELTA_BYTE_ARRAY" in c["encodings"] and not GPU_DBA:
            continue
        chunks.append(ch)
        exp.append(e)
    # SNAPPY chunks are decompressed on the device straight into the batch (pqg_snappy_decompress)
    cols, st = decoder.decode(decoder.upload_chunks(chunks))
    for col, e, ch in zip(cols, exp, chunks):
        assert_same(col.numpy(), e, ch.physical_type)
