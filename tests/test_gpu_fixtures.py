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


def test_gpu_decodes_raw_chunk_bytes(decoder):
    """File bytes in: every UNCOMPRESSED fixture chunk's raw bytes (page headers included) go to the
    device as they sit in the file; pqg_frame_chunk (with CRC verification) + pqg_pages_from_headers
    describe the pages, and one pqg_decode over all chunks yields the expected values."""
    import ctypes as C
    import os

    import fixtures
    from pqgpu import framing, native
    from tools.synth import writer
    L = native.lib()
    pieces, descs, columns, slots, exp, ptypes = [], [], [], [], [], []
    pos = 0
    for name, c in CASES:
        ch, e = load_chunk(name, c)
        if fixtures.is_compressed(ch) or c["num_values"] == 0:
            continue
        buf = np.fromfile(os.path.join(fixtures.GOLDEN, name + ".parquet"), dtype=np.uint8).tobytes()
        raw = buf[c["start"]: c["start"] + c["length"]]
        rc, st, hdrs = framing.frame_chunk_native(raw, c["num_values"], verify_crc=True)
        assert rc == abi.OK, st.message
        base = (pos + 15) // 16 * 16
        arr = (abi.PageHeader * len(hdrs))(*hdrs)
        col = abi.ColumnDesc()
        col.dict_offset = -1
        pages = (abi.PageDesc * len(hdrs))()
        n = C.c_int(0)
        rc = L.pqg_pages_from_headers(C.addressof(arr), len(hdrs), abi.CODEC_UNCOMPRESSED, base, len(columns), C.byref(col),
                                      C.addressof(pages), len(hdrs), C.byref(n), C.byref(st))
        assert rc == abi.OK, st.message
        descs += [bytes(pages[k]) for k in range(n.value)]
        columns.append(dict(physical_type=ch.physical_type, type_length=ch.type_length, max_rep=ch.max_rep,
                            max_def=ch.max_def, dict_offset=col.dict_offset, dict_size=col.dict_size,
                            dict_num_values=col.dict_num_values, dict_encoding=col.dict_encoding))
        slots.append(sum(pages[k].num_values for k in range(n.value)))
        pieces.append((base, raw))
        pos = base + len(raw)
        exp.append(e)
        ptypes.append(ch.physical_type)
    data = np.zeros(pos + writer.PAD, dtype=np.uint8)
    for base, raw in pieces:
        data[base: base + len(raw)] = np.frombuffer(raw, dtype=np.uint8)
    page_arr = np.frombuffer(b"".join(descs), dtype=abi.PAGE_DTYPE).copy()
    batch = writer.PageBatch(data=data, pages=page_arr, columns=columns, chunks=[],
                             page_slot_offsets=np.zeros(len(page_arr), np.int64), column_slots=slots,
                             column_values=[len(e) for e in exp])
    cols, st = decoder.decode(decoder.upload(batch))
    assert len(cols) >= 20
    for col, e, pt in zip(cols, exp, ptypes):
        assert_same(col.numpy(), e, pt)
