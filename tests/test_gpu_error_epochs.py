"""Error words across launches of one plan (pqg_plan_launch re-runs).

Error words and the error counter are tagged with the plan's launch epoch instead of being
reset before every launch (pqgpu_internal.h ErrCount). These tests flip one device byte between
launches of the same plan so that an error appears, disappears and reappears, including across
the epoch wrap (65,535 launches), and check each launch's status against the oracle — the
reference's DictionaryValuesReader throws on the bad id (`DictionaryValuesReader.java:79-84`,
`PlainValuesDictionary.PlainLongDictionary.decodeToLong`) and reads the good page cleanly.
"""
import numpy as np
import pytest
import torch

from oracle import pqref
from pqgpu import abi
from tools.synth import writer

from helpers import make, zipf_dict_column

pytestmark = pytest.mark.gpu


def _varint(b, i):
    v = s = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << s
        s += 7
        if not c & 0x80:
            return v, i


def _good_and_bad():
    ch = make(abi.INT64, zipf_dict_column(8000, card=100, a=1.5, seed=5), abi.RLE_DICTIONARY, page_rows=1000)
    good = writer.build_batch([ch])
    for p, pg in enumerate(ch.pages):
        body = bytes(pg.body)
        w = body[0]
        hdr, i = _varint(body, 1)
        if hdr & 1 == 0 and w == 7:  # first run is an RLE run: its value follows in 1 byte (w = 7)
            pg.body = body[:i] + bytes([0x7F]) + body[i + 1:]  # id 127 >= 100 entries
            bad = writer.build_batch([ch])
            diff = np.flatnonzero(good.data != bad.data)
            assert diff.size == 1
            return good, bad, int(diff[0]), p
    pytest.skip("no page starts with an RLE run")


def test_error_epochs_across_relaunches(decoder):
    good, bad, off, page = _good_and_bad()
    ref_good, ref_bad = pqref.decode_batch(good), pqref.decode_batch(bad)
    assert ref_good.code == 0 and ref_bad.code != 0 and ref_bad.status[1] == page
    dbatch = decoder.upload(good)
    plan = decoder.plan(dbatch)
    good_byte, bad_byte = int(good.data[off]), int(bad.data[off])

    def run(byte, n=1):
        dbatch.bytes[off] = byte
        torch.cuda.synchronize()
        for _ in range(n):
            plan.launch()
        rc, st = plan.sync()
        return rc, (int(st.code), int(st.page), int(st.value_index))

    try:
        assert run(bad_byte) == (ref_bad.code, ref_bad.status)
        assert run(good_byte) == (0, ref_good.status)       # stale words of the last launch are ignored
        assert run(bad_byte, 3) == (ref_bad.code, ref_bad.status)
        assert run(good_byte, 70000) == (0, ref_good.status)  # crosses the 16-bit epoch wrap
        assert run(bad_byte) == (ref_bad.code, ref_bad.status)
        assert run(good_byte) == (0, ref_good.status)
        got = plan.columns[0].numpy()
        assert np.array_equal(got.view(np.uint64), ref_good.columns[0]["values"].view(np.uint64))
    finally:
        plan.close()
