"""C4 (BASELINE.json configs[3]): TPC-H lineitem-shaped 16 columns, row groups of ~1M rows.

Columns, all REQUIRED (lineitem is NOT NULL), parquet-mr V1 pages of 20,000 values, uncompressed;
the encodings SURVEY.md §8d names for C4:

  0 l_orderkey      INT64       DELTA_BINARY_PACKED   sorted; 1-7 lines per order; sparse keys (8 of 32)
  1 l_partkey       INT64       DELTA_BINARY_PACKED   uniform [1, 33,333,333]
  2 l_suppkey       INT64       DELTA_BINARY_PACKED   uniform [1, 1,666,667]
  3 l_linenumber    INT32       RLE_DICTIONARY        1..lines of the order (7 entries, short runs)
  4 l_quantity      DOUBLE      PLAIN                 1..50
  5 l_extendedprice DOUBLE      PLAIN                 quantity x part price
  6 l_discount      DOUBLE      PLAIN                 0.00..0.10
  7 l_tax           DOUBLE      PLAIN                 0.00..0.08
  8 l_returnflag    BYTE_ARRAY  RLE_DICTIONARY        R / A / N (by receipt date)
  9 l_linestatus    BYTE_ARRAY  RLE_DICTIONARY        O / F (by ship date)
 10 l_shipdate      INT32       DELTA_BINARY_PACKED   days since 1970: order date + 1..121
 11 l_commitdate    INT32       DELTA_BINARY_PACKED   order date + 30..90
 12 l_receiptdate   INT32       DELTA_BINARY_PACKED   ship date + 1..30
 13 l_shipinstruct  BYTE_ARRAY  RLE_DICTIONARY        4 values
 14 l_shipmode      BYTE_ARRAY  RLE_DICTIONARY        7 values
 15 l_comment       BYTE_ARRAY  PLAIN                 10..43 random characters

The same generator makes every row group from its seed, so a run can synthesize a few distinct
row groups and lay them out repeatedly (the decode of each copy is independent work).
"""
import numpy as np

from pqgpu import abi
from tools.synth import writer
from workloads import Expected, Workload, binary_take

COLUMNS = [
    ("l_orderkey", abi.INT64, abi.DELTA_BINARY_PACKED), ("l_partkey", abi.INT64, abi.DELTA_BINARY_PACKED),
    ("l_suppkey", abi.INT64, abi.DELTA_BINARY_PACKED), ("l_linenumber", abi.INT32, abi.RLE_DICTIONARY),
    ("l_quantity", abi.DOUBLE, abi.PLAIN), ("l_extendedprice", abi.DOUBLE, abi.PLAIN),
    ("l_discount", abi.DOUBLE, abi.PLAIN), ("l_tax", abi.DOUBLE, abi.PLAIN),
    ("l_returnflag", abi.BYTE_ARRAY, abi.RLE_DICTIONARY), ("l_linestatus", abi.BYTE_ARRAY, abi.RLE_DICTIONARY),
    ("l_shipdate", abi.INT32, abi.DELTA_BINARY_PACKED), ("l_commitdate", abi.INT32, abi.DELTA_BINARY_PACKED),
    ("l_receiptdate", abi.INT32, abi.DELTA_BINARY_PACKED), ("l_shipinstruct", abi.BYTE_ARRAY, abi.RLE_DICTIONARY),
    ("l_shipmode", abi.BYTE_ARRAY, abi.RLE_DICTIONARY), ("l_comment", abi.BYTE_ARRAY, abi.PLAIN),
]
SHIPINSTRUCT = [b"DELIVER IN PERSON", b"COLLECT COD", b"NONE", b"TAKE BACK RETURN"]
SHIPMODE = [b"REG AIR", b"AIR", b"RAIL", b"SHIP", b"TRUCK", b"MAIL", b"FOB"]
DAY0, DAY1 = 8035, 10591        # 1992-01-01 .. 1998-12-31 (days since 1970-01-01)
CUTOFF = 9298                   # 1995-06-17


def _dict_column(ptype, words_or_vals, ids):
    """Dictionary column from raw ids: ids renumbered in first-appearance order (what
    DictionaryValuesWriter assigns), PLAIN dictionary page, RLE/bit-packed hybrid ids."""
    ids_fa, order = writer.first_appearance_ids(ids)
    if ptype == abi.BYTE_ARRAY:
        words = [words_or_vals[o] for o in order]
        dv = writer.BinaryValues(np.concatenate([[0], np.cumsum([len(w) for w in words])]),
                                 np.frombuffer(b"".join(words), dtype=np.uint8))
        ch = writer.write_dict_column_from_ids(abi.BYTE_ARRAY, dv, ids_fa)
        return ch, binary_take(words_or_vals, ids)
    vals = np.asarray(words_or_vals)
    ch = writer.write_dict_column_from_ids(ptype, vals[order], ids_fa)
    return ch, vals[ids]


def make_row_group(n, seed, order_base=0):
    """One lineitem row group of n rows -> (16 ColumnChunks, 16 Expected)."""
    rng = np.random.default_rng(seed)
    lines = rng.integers(1, 8, size=n // 2 + 8)
    cut = int(np.searchsorted(np.cumsum(lines), n)) + 1
    lines = lines[:cut]
    lines[-1] -= int(lines.sum()) - n
    n_ord = lines.size
    o = np.arange(order_base, order_base + n_ord, dtype=np.int64)
    okey_o = (o // 8) * 32 + (o % 8) + 1
    odate_o = rng.integers(DAY0, DAY1 - 151, size=n_ord)
    okey = np.repeat(okey_o, lines)
    odate = np.repeat(odate_o, lines)
    first = np.repeat(np.cumsum(lines) - lines, lines)
    linenumber = (np.arange(n) - first + 1).astype(np.int32)
    partkey = rng.integers(1, 33_333_334, size=n, dtype=np.int64)
    suppkey = rng.integers(1, 1_666_668, size=n, dtype=np.int64)
    qty = rng.integers(1, 51, size=n).astype(np.float64)
    price = (90000 + (partkey // 10) % 20001 + 100 * (partkey % 1000)) / 100.0
    extprice = np.round(qty * price, 2)
    disc = rng.integers(0, 11, size=n) / 100.0
    tax = rng.integers(0, 9, size=n) / 100.0
    ship = (odate + rng.integers(1, 122, size=n)).astype(np.int32)
    commit = (odate + rng.integers(30, 91, size=n)).astype(np.int32)
    receipt = (ship + rng.integers(1, 31, size=n)).astype(np.int32)
    rf = np.where(receipt <= CUTOFF, rng.integers(0, 2, size=n), 2)          # R, A | N
    ls = np.where(ship > CUTOFF, 0, 1)                                         # O | F
    si = rng.integers(0, 4, size=n)
    sm = rng.integers(0, 7, size=n)
    comment = writer.BinaryValues.random(n, 10, 43, seed=seed + 7, alphabet=b"abcdefghijklmnopqrstuvwxyz ,.")

    chunks, exp = [], []

    def plain_or_delta(ptype, enc, v):
        chunks.append(writer.write_column_chunk(ptype, v, enc))
        exp.append(Expected(v))

    def dictionary(ptype, vocab, ids):
        ch, v = _dict_column(ptype, vocab, ids)
        chunks.append(ch)
        exp.append(Expected(v))

    plain_or_delta(abi.INT64, abi.DELTA_BINARY_PACKED, okey)
    plain_or_delta(abi.INT64, abi.DELTA_BINARY_PACKED, partkey)
    plain_or_delta(abi.INT64, abi.DELTA_BINARY_PACKED, suppkey)
    dictionary(abi.INT32, np.arange(1, 8, dtype=np.int32), linenumber - 1)
    for v in (qty, extprice, disc, tax):
        plain_or_delta(abi.DOUBLE, abi.PLAIN, v)
    dictionary(abi.BYTE_ARRAY, [b"R", b"A", b"N"], rf)
    dictionary(abi.BYTE_ARRAY, [b"O", b"F"], ls)
    for v in (ship, commit, receipt):
        plain_or_delta(abi.INT32, abi.DELTA_BINARY_PACKED, v)
    dictionary(abi.BYTE_ARRAY, SHIPINSTRUCT, si)
    dictionary(abi.BYTE_ARRAY, SHIPMODE, sm)
    chunks.append(writer.write_column_chunk(abi.BYTE_ARRAY, comment, abi.PLAIN))
    exp.append(Expected(comment))
    for ch, e in zip(chunks, exp):
        if ch.values is None:
            ch.values = e.values
    return chunks, exp, n_ord


def make_c4(rows, rg_rows=1_000_000, seed=1000):
    """A single batch of rows // rg_rows row groups (tests; the bench lays out copies itself)."""
    chunks, exp = [], []
    base = 0
    for g in range(max(1, rows // rg_rows)):
        c, e, n_ord = make_row_group(min(rg_rows, rows), seed + g, base)
        base += n_ord
        chunks += c
        exp += e
    return Workload("c4_lineitem", chunks, exp)


class Shard:
    """One rank's share of the C4 table: `rows` rows in total in row groups of `rg_rows`, split over
    `world` ranks by encoded bytes (pqgpu.dist.shard_row_groups, the Hadoop row-group split,
    ParquetInputFormat.java:350,786). T distinct synthetic row groups are laid out repeatedly (row
    group g = template g mod T): every copy's pages are decoded, none is skipped. Dictionary columns
    are one pqg column per row group (each row group has its own dictionary); the other columns
    decode every row group of the rank into one rank-wide column, back to back."""

    def __init__(self, rows, world=1, rank=0, templates=4, rg_rows=1_000_000, keep=None):
        import copy

        from pqgpu import dist as pdist
        self.rg_rows = rg_rows
        self.n_rg = max(1, rows // rg_rows)
        self.T = min(templates, self.n_rg)
        self.templates, base = [], 0
        for t in range(self.T):
            ch, ex, n_ord = make_row_group(rg_rows, 1000 + t, base)
            base += n_ord
            self.templates.append((ch, ex))
        tsize = [sum(len(p.body) for c in ch for p in c.pages) for ch, _ in self.templates]
        self.shards = pdist.shard_row_groups([tsize[g % self.T] for g in range(self.n_rg)], world)
        self.mine = self.shards[rank]
        # keep: the lineitem columns decoded (diagnostics: a subset's kernels without the others' overlap)
        self.keep = list(range(16)) if keep is None else sorted(keep)
        self.chunks = []
        for g in self.mine:
            for k, c in enumerate(self.templates[g % self.T][0]):
                if k not in self.keep:
                    continue
                cc = copy.copy(c)
                cc.column_index = (k, g) if c.dict_page is not None else (k, -1)
                self.chunks.append(cc)
        self.batch = writer.build_batch(self.chunks)
        self.col_of = {}
        for c in self.chunks:
            self.col_of.setdefault(c.column_index, len(self.col_of))

    def column(self, k, g):
        """pqg column index of lineitem column k in row group g, and whether it is rank-wide."""
        merged = (k, -1) in self.col_of
        return (self.col_of[(k, -1)] if merged else self.col_of[(k, g)]), merged

    def verify(self, cols, device, what):
        """Every row group x column slice of the decoded columns == its template's generated values
        (compared on the device)."""
        import torch
        exp_dev = {}
        pos = {k: 0 for k in self.keep}
        n = self.rg_rows
        for g in self.mine:
            t = g % self.T
            for k in self.keep:
                ci, merged = self.column(k, g)
                col = cols[ci]
                ex = self.templates[t][1][k]
                if (t, k) not in exp_dev:
                    if isinstance(ex.values, writer.BinaryValues):
                        exp_dev[(t, k)] = (torch.from_numpy(ex.values.offsets).to(device),
                                           torch.from_numpy(ex.values.data).to(device))
                    else:
                        exp_dev[(t, k)] = torch.from_numpy(np.ascontiguousarray(ex.values).view(np.uint8)).to(device)
                e = exp_dev[(t, k)]
                r0 = pos[k] if merged else 0
                if isinstance(e, tuple):
                    offs = col.offsets()[r0:r0 + n + 1]
                    b0 = int(offs[0].item())
                    assert torch.equal(offs - b0, e[0]), f"{what}: row group {g} column {k} offsets"
                    assert torch.equal(col.binary_data[b0:b0 + e[1].numel()], e[1]), f"{what}: rg {g} col {k} bytes"
                else:
                    w = e.numel() // n
                    assert torch.equal(col.values[r0 * w:(r0 + n) * w], e), f"{what}: row group {g} column {k}"
                if merged:
                    pos[k] += n
        for k in self.keep:  # every rank-wide column holds exactly its row groups' values
            ci, merged = self.column(k, self.mine[0]) if self.mine else (None, False)
            if merged:
                assert cols[ci].n_values == len(self.mine) * n, f"{what}: column {k} value count"
