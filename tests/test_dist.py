"""Multi-rank path on CPU (gloo, world_size 2): row-group sharding + the all-gather
concatenation. The per-rank decode here is the oracle (the GPU decode runs in the
-m gpu tests); what is tested is the sharding / offset / gather logic."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from pqgpu import abi, dist as pdist
from tools.synth import writer


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _row_groups():
    rng = np.random.default_rng(3)
    rgs = []
    for k in range(7):
        n = int(rng.integers(1000, 20000))
        vals = rng.integers(0, 300, size=n)[np.repeat(np.arange(n // 10 + 1), 10)[:n]].astype(np.int64) * (k + 1)
        rgs.append(writer.write_column_chunk(abi.INT64, vals, abi.RLE_DICTIONARY, page_rows=4000))
    return rgs


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from oracle import pqref
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rgs = _row_groups()
    sizes = [sum(len(p.body) for p in ch.pages) for ch in rgs]
    rows = [len(ch.values) for ch in rgs]
    shards = pdist.shard_row_groups(sizes, world)
    mine = shards[rank]
    local = []
    for i in mine:
        res = pqref.decode_batch(writer.build_batch([rgs[i]]))
        assert res.code == 0
        local.append(res.columns[0]["values"])
    local = torch.from_numpy(np.concatenate(local) if local else np.zeros(0, np.int64))
    full = pdist.gather_column(local, mine, shards, rows)
    expect = np.concatenate([ch.values for ch in rgs])
    ok = bool(np.array_equal(full.numpy(), expect))
    # BYTE_ARRAY: byte-total all-gather + offset rebase (PLAIN strings of 0-40 bytes per row group)
    brgs = _binary_row_groups()
    bshards = pdist.shard_row_groups([sum(len(p.body) for p in ch.pages) for ch in brgs], world)
    offs, data = [np.zeros(1, np.int64)], []
    for i in bshards[rank]:
        res = pqref.decode_batch(writer.build_batch([brgs[i]]))
        assert res.code == 0
        vals = res.columns[0]["values"]
        lens = np.array([len(v) for v in vals], dtype=np.int64)
        offs.append(offs[-1][-1] + np.cumsum(lens))
        data.append(np.frombuffer(b"".join(vals), dtype=np.uint8))
    loff = torch.from_numpy(np.concatenate(offs))
    ldata = torch.from_numpy(np.concatenate(data) if data else np.zeros(0, np.uint8))
    foff, fdata = pdist.gather_binary(loff, ldata, bshards[rank], bshards, [len(ch.values) for ch in brgs])
    allv = [bytes(v) for ch in brgs for v in ch.values]
    exp_off = np.concatenate([[0], np.cumsum([len(v) for v in allv])])
    ok_b = bool(np.array_equal(foff.numpy(), exp_off)) and fdata.numpy().tobytes() == b"".join(allv)
    ok_c4 = _c4_gather(rank, world)
    q.put((rank, ok and ok_b and ok_c4, [len(s) for s in shards], [len(s) for s in bshards]))
    dist.destroy_process_group()


def _c4_gather(rank, world):
    """C4 lineitem row groups (small ones: 5 x 20,000 rows) sharded over the ranks, each rank's share
    decoded (the oracle here; the GPU decode of the same row groups runs in the -m gpu tests), then
    l_orderkey (int64) and l_comment (BYTE_ARRAY) gathered into the full columns on every rank."""
    import lineitem as LI
    from oracle import pqref
    rgs, base = [], 0
    for g in range(5):
        ch, ex, n_ord = LI.make_row_group(20_000, 500 + g, base)
        base += n_ord
        rgs.append((ch, ex))
    sizes = [sum(len(p.body) for c in ch for p in c.pages) for ch, _ in rgs]
    shards = pdist.shard_row_groups(sizes, world)
    mine = shards[rank]
    keys, offs, data = [], [np.zeros(1, np.int64)], []
    for g in mine:
        r = pqref.decode_batch(writer.build_batch([rgs[g][0][0], rgs[g][0][15]]))
        assert r.code == 0
        keys.append(r.columns[0]["values"])
        vals = r.columns[1]["values"]
        offs.append(offs[-1][-1] + np.cumsum([len(v) for v in vals]))
        data.append(np.frombuffer(b"".join(vals), dtype=np.uint8))
    counts = [20_000] * 5
    full = pdist.gather_column(torch.from_numpy(np.concatenate(keys) if keys else np.zeros(0, np.int64)), mine, shards,
                               counts)
    ok = np.array_equal(full.numpy(), np.concatenate([ex[0].values for _, ex in rgs]))
    foff, fdata = pdist.gather_binary(torch.from_numpy(np.concatenate(offs)),
                                      torch.from_numpy(np.concatenate(data) if data else np.zeros(0, np.uint8)),
                                      mine, shards, counts)
    exp_off, exp_data = [np.zeros(1, np.int64)], []
    for _, ex in rgs:
        v = ex[15].values
        exp_off.append(exp_off[-1][-1] + v.offsets[1:])
        exp_data.append(v.data[: v.offsets[-1]])
    ok = ok and np.array_equal(foff.numpy(), np.concatenate(exp_off))
    return bool(ok and np.array_equal(fdata.numpy(), np.concatenate(exp_data)))


def _binary_row_groups():
    rng = np.random.default_rng(5)
    rgs = []
    for k in range(5):
        n = int(rng.integers(0 if k == 2 else 100, 3000))
        vals = writer.BinaryValues.random(n, 0, 40, seed=100 + k)
        ch = writer.write_column_chunk(abi.BYTE_ARRAY, vals, abi.PLAIN, page_rows=700)
        ch.values = [vals[i] for i in range(n)]
        rgs.append(ch)
    return rgs


def test_shard_row_groups_contiguous_and_balanced():
    sizes = [10, 9, 8, 1, 1, 1, 7, 3]
    sh = pdist.shard_row_groups(sizes, 3)
    assert sum(sh, []) == list(range(8))               # contiguous ranges in file order, rank order
    loads = [sum(sizes[i] for i in s) for s in sh]
    assert max(loads) - min(loads) <= max(sizes)        # balanced within one row group
    # the configured C4 shard: 1,000 near-equal row groups over 8 ranks -> 125 each
    rng = np.random.default_rng(0)
    sh8 = pdist.shard_row_groups(75_330_000 + rng.integers(-20_000, 20_000, size=1000), 8)
    assert [len(s) for s in sh8] == [125] * 8
    assert pdist.shard_row_groups([], 4) == [[], [], [], []]
    assert sum(pdist.shard_row_groups([5, 5], 4), []) == [0, 1]


def test_row_group_offsets():
    assert list(pdist.row_group_offsets([5, 0, 7])) == [0, 5, 5]


def test_gather_world2_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] for r in res), res
    assert all(p.exitcode == 0 for p in procs)
