"""GPU parity of the window walks (decode_levels_bl for level sections, dict_walk_ls for dictionary
ids) on hand-built RLE / bit-packed hybrid sections that the parquet-mr writer never produces but the
reader accepts (RunLengthBitPackingHybridDecoder.readNext,
parquet-column/.../rle/RunLengthBitPackingHybridDecoder.java:80-109):

  * bit-packed runs longer than 63 groups (other writers; runs whose data passes the walk's staged
    bytes), RLE runs of hundreds of thousands of values (one header for a whole page), pages larger
    than the walk's LDS segment, widths 1..8 for levels and 0..32 for dictionary ids;
  * the headers outside the walks' branch-free pre-decode (scalar slow path): an RLE level value wider
    than the width (read unmasked), an RLE run of count 0 (the reader repeats its value for the rest of
    the page), a section that ends before the page's slots / values do.

Every case is compared with the oracle (values bit for bit, levels, per-page counts, first error).
"""
import numpy as np
import pytest

from oracle import pqref
from pqgpu import abi
from tools.synth import writer
from tools.synth.writer import ColumnChunk, Page

from helpers import assert_same

pytestmark = pytest.mark.gpu


def uvarint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def pack_lsb(vals, w):
    """LSB-first bit packing of len(vals) values (a multiple of 8) at width w."""
    if w == 0:
        return b""
    bits = 0
    for i, v in enumerate(vals):
        bits |= (int(v) & ((1 << w) - 1)) << (i * w)
    return bits.to_bytes(len(vals) * w // 8, "little")


def hybrid(runs, w):
    """Section bytes and decoded values of [('rle', count, value) | ('packed', values)]."""
    out, vals = bytearray(), []
    nb = (w + 7) // 8
    for r in runs:
        if r[0] == "rle":
            _, c, v = r
            out += uvarint(c << 1) + int(v).to_bytes(nb, "little")
            vals += [v] * c
        else:
            pv = list(r[1])
            assert len(pv) % 8 == 0
            out += uvarint(((len(pv) // 8) << 1) | 1) + pack_lsb(pv, w)
            vals += pv
    return bytes(out), vals


def read_hybrid(sec, w, n):
    """The values RunLengthBitPackingHybridDecoder.readInt returns for n reads of `sec`
    (readNext :80-109: RLE values unmasked, a 0-count RLE run repeats forever, a packed run reads
    what is left of the section), up to the first read that throws."""
    out, p, nb = [], 0, (w + 7) // 8
    while len(out) < n:
        if p >= len(sec):
            break
        h, s = 0, 0
        while p < len(sec):
            b = sec[p]
            p += 1
            h |= (b & 0x7F) << s
            s += 7
            if b < 0x80:
                break
        if h & 1:
            g = h >> 1
            data = sec[p:p + g * w].ljust(g * w, b"\0")
            p = min(p + g * w, len(sec))
            bits = int.from_bytes(data, "little")
            out += [(bits >> (i * w)) & ((1 << w) - 1) for i in range(8 * g)]
        else:
            v = int.from_bytes(sec[p:p + nb], "little")
            p += nb
            c = h >> 1
            out += [v] * (c if c else n - len(out))
    return out[:n]


def random_runs(rng, n, w, max_group=300, max_rle=5000, p_rle=0.5):
    runs, total = [], 0
    top = (1 << w) - 1
    while total < n:
        if rng.random() < p_rle:
            c = int(rng.integers(1, max_rle + 1))
            runs.append(("rle", c, int(rng.integers(0, top + 1))))
        else:
            g = int(rng.integers(1, max_group + 1))
            runs.append(("packed", rng.integers(0, top + 1, size=8 * g).tolist()))
        total += runs[-1][1] if runs[-1][0] == "rle" else len(runs[-1][1])
    return runs


def level_chunk(sections, max_def, seed=0):
    """An optional INT64 column of V2 pages whose definition-level sections are the given bytes;
    each entry: (section bytes, slots of the page, its levels as the reader decodes them)."""
    rng = np.random.default_rng(seed)
    ch = ColumnChunk(physical_type=abi.INT64, max_def=max_def)
    total = 0
    for sec, n_slots, levels in sections:
        nn = int(np.count_nonzero(np.asarray(levels[:n_slots]) == max_def))
        data = rng.integers(-2**40, 2**40, size=nn).astype(np.int64).tobytes()
        pg = Page(body=sec + data, num_values=n_slots, encoding=abi.PLAIN, version=2)
        pg.rl_byte_length, pg.dl_byte_length = 0, len(sec)
        ch.pages.append(pg)
        total += nn
    ch.n_values_hint = total
    return ch


def run_both(decoder, chunks):
    batch = writer.build_batch(chunks)
    ref = pqref.decode_batch(batch)
    dcols, st = decoder.decode(decoder.upload(batch), check=False)
    assert (int(st.code), int(st.page), int(st.value_index)) == ref.status, \
        f"gpu status {st.code, st.page, st.value_index} {st.message} vs oracle {ref.status}"
    if ref.code:
        return ref
    for i, cd in enumerate(batch.columns):
        col = dcols[i]
        assert col.n_values == ref.columns[i]["n_values"]
        assert_same(col.numpy(), ref.columns[i]["values"], cd["physical_type"])
        if cd["max_def"] > 0:
            assert np.array_equal(col.def_levels[:batch.column_slots[i]].cpu().numpy(), ref.columns[i]["def_levels"])
    return ref


# ---- level sections -------------------------------------------------------------------------------

@pytest.mark.parametrize("max_def", [1, 3, 5, 15, 31, 63, 127, 254])
@pytest.mark.parametrize("shape", ["long_packed", "long_rle", "mixed"])
def test_levels_hand_built_runs(decoder, max_def, shape):
    """Packed runs of up to 300 groups (an 8-bit-level page: 2,400 data bytes in one run; max_def 254 is the
    device limit, pqg_plan_create: 255 is UNSUPPORTED), RLE runs of
    up to 5,000 slots, pages of 30,000-60,000 slots, every width 1..8."""
    w = int(max_def).bit_length()
    rng = np.random.default_rng(max_def * 3 + len(shape))
    secs = []
    for k in range(4):
        n = int(rng.integers(30_000, 60_000))
        if shape == "long_packed":
            runs = random_runs(rng, n, w, max_group=300, max_rle=40, p_rle=0.2)
        elif shape == "long_rle":
            runs = random_runs(rng, n, w, max_group=3, max_rle=5000, p_rle=0.7)
        else:
            runs = random_runs(rng, n, w, max_group=2, max_rle=9, p_rle=0.5)
        sec, lv = hybrid(runs, w)
        secs.append((sec, n, lv))
    run_both(decoder, [level_chunk(secs, max_def, seed=max_def)])


@pytest.mark.parametrize("max_def", [1, 3])
def test_levels_one_rle_run_per_page(decoder, max_def):
    """Pages without nulls: one RLE header for 300,000 slots (the whole wave fills the level image,
    several images per page)."""
    w = int(max_def).bit_length()
    secs = []
    for n in (300_000, 70_001, 16):
        sec, lv = hybrid([("rle", n, max_def)], w)
        secs.append((sec, n, lv))
    # and a page of nulls
    sec, lv = hybrid([("rle", 50_000, 0)], w)
    secs.append((sec, 50_000, lv))
    run_both(decoder, [level_chunk(secs, max_def)])


def test_levels_large_random_page(decoder):
    """200,000 random 2-bit levels in one page (mostly bit-packed): many level images and
    super-windows per page."""
    rng = np.random.default_rng(5)
    lv = rng.integers(0, 4, size=200_000).astype(np.uint8)
    sec = writer.rle_encode_levels(lv, 2)
    run_both(decoder, [level_chunk([(sec, lv.size, lv.tolist())], 3)])


@pytest.mark.parametrize("case", ["wide_rle_value", "zero_count_rle", "short_section", "truncated_group"])
def test_levels_slow_path_headers(decoder, case):
    """Sections with headers outside the pre-decode's fast path: its result (levels, counts, error
    at the oracle's slot) must be the same."""
    rng = np.random.default_rng(len(case))
    w, max_def = 2, 3
    base = random_runs(rng, 20_000, w, max_group=10, max_rle=30)
    if case == "wide_rle_value":
        runs = base[:40] + [("rle", 17, 2)] + base[40:]
        sec, lv = hybrid(runs, w)
        sec = bytearray(sec)
        # the RLE value byte of the inserted run rewritten to 7 (> max level, read unmasked)
        s1, _ = hybrid(base[:40], w)
        sec[len(s1) + 1] = 7
        sec = bytes(sec)
        n = len(lv)
    elif case == "zero_count_rle":
        s1, l1 = hybrid(base[:30], w)
        sec = s1 + uvarint(0) + bytes([3])
        n = len(l1) + 5000
    elif case == "short_section":
        sec, lv = hybrid(base, w)
        n = len(lv) + 4000
    else:  # the last packed group's bytes cut: the reader reads what is left, the rest is 0
        sec, lv = hybrid(base + [("packed", [1] * 64)], w)
        sec = sec[:-5]
        n = len(lv)
    # the page's data: one value per slot the reader decodes as non-null before any level error
    run_both(decoder, [level_chunk([(sec, n, read_hybrid(sec, w, n))], max_def)])


# ---- dictionary-id sections -------------------------------------------------------------------------

def dict_chunk(pages, card, physical_type=abi.INT64, seed=0):
    """An RLE_DICTIONARY column: pages = [(bit width, runs)], ids < card."""
    rng = np.random.default_rng(seed)
    dvals = rng.integers(-2**62, 2**62, size=card).astype(np.int64)
    ch = ColumnChunk(physical_type=physical_type)
    ch.dict_page = writer.plain_encode(dvals, physical_type)
    ch.dict_num_values = card
    total = 0
    for w, runs in pages:
        sec, ids = hybrid(runs, w)
        ch.pages.append(Page(body=bytes([w]) + sec, num_values=len(ids), encoding=abi.RLE_DICTIONARY))
        total += len(ids)
    ch.n_values_hint = total
    return ch


@pytest.mark.parametrize("w", [0, 1, 3, 7, 8, 9, 13, 16, 17, 24, 25, 31, 32])
def test_dict_ids_hand_built_widths(decoder, w):
    """Id sections at every byte-size class of the RLE value (1-4 bytes), with declared widths
    larger than the dictionary needs (the reader takes the page's width byte as is), packed runs of
    up to 200 groups and RLE runs of up to 3,000 values."""
    card = 37
    rng = np.random.default_rng(w + 100)
    pages = []
    for k in range(3):
        runs, total = [], 0
        while total < 25_000:
            if rng.random() < 0.5:
                c = int(rng.integers(1, 3000))
                runs.append(("rle", c, int(rng.integers(0, card)) if w else 0))  # (w = 0: no value bytes)
                total += c
            else:
                g = int(rng.integers(1, 200))
                runs.append(("packed", rng.integers(0, card if w else 1, size=8 * g).tolist()))
                total += 8 * g
        pages.append((w, runs))
    run_both(decoder, [dict_chunk(pages, card, seed=w)])


@pytest.mark.parametrize("case", ["zero_count_rle", "short_section", "id_past_dictionary"])
def test_dict_ids_handed_back(decoder, case):
    """Sections dict_walk_sp hands to the window walk (0-count RLE run: the value repeats for the
    rest of the page; a section shorter than the page's values) and an id past the dictionary
    (reported by the expansion at its value)."""
    rng = np.random.default_rng(7)
    card, w = 20, 5
    runs = [("packed", rng.integers(0, card, size=8 * 5).tolist()), ("rle", 100, 3)] * 30
    sec, ids = hybrid(runs, w)
    n = len(ids)
    if case == "zero_count_rle":
        sec = sec + uvarint(0) + bytes([4])
        n += 777
    elif case == "short_section":
        n += 500
    else:
        sec, ids = hybrid(runs + [("rle", 9, card + 2)], w)
        n = len(ids)
    ch = ColumnChunk(physical_type=abi.INT64)
    dvals = rng.integers(-2**62, 2**62, size=card).astype(np.int64)
    ch.dict_page = writer.plain_encode(dvals, abi.INT64)
    ch.dict_num_values = card
    ch.pages.append(Page(body=bytes([w]) + sec, num_values=n, encoding=abi.RLE_DICTIONARY))
    ch.n_values_hint = n
    run_both(decoder, [ch])
