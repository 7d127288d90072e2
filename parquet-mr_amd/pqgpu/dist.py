"""Row-group sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

A row group's column chunks decode with no cross-chunk state, so ranks decode
disjoint row groups with no data-path collective. The only exchange is the final column
concatenation, when a consumer wants the full column on every rank (all-gather over RCCL):

  * fixed-width columns: output offsets of each row group are prefix sums of footer row counts,
    so the decoded slices are all-gathered as they are;
  * BYTE_ARRAY columns: one all-gather of every rank's byte total, an exclusive scan of them for
    the ranks' byte bases, then the offsets and value bytes are all-gathered and each row group's
    offsets rebased onto the concatenated byte buffer.

Reference parallelism being restated: Hadoop InputSplits at row-group granularity
(parquet-hadoop/src/main/java/org/apache/parquet/hadoop/ParquetInputFormat.java: getSplits :350,
generateSplits :786).
"""
import numpy as np
import torch
import torch.distributed as dist


def shard_row_groups(sizes, world):
    """Greedy longest-processing-time assignment of row groups (by encoded bytes) to ranks.
    Returns, per rank, the sorted list of its row-group indices."""
    order = sorted(range(len(sizes)), key=lambda i: (-sizes[i], i))
    load = [0] * world
    out = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        out[r].append(i)
        load[r] += sizes[i]
    return [sorted(x) for x in out]


def row_group_offsets(row_counts):
    """First output row of each row group in the concatenated column."""
    return np.concatenate([[0], np.cumsum(np.asarray(row_counts, dtype=np.int64))])[:-1]


def _on_backend(t, group):
    """gloo collectives run on host tensors; RCCL (backend "nccl") on device tensors."""
    return t.cpu() if dist.get_backend(group) == "gloo" else t


def _all_gather_padded(t, maxlen, group):
    """All-gather 1-D tensors of different lengths (each padded to maxlen)."""
    world = dist.get_world_size(group)
    src = _on_backend(t, group)
    buf = torch.zeros(maxlen, dtype=src.dtype, device=src.device)
    buf[: src.numel()] = src
    out = torch.empty(world * maxlen, dtype=src.dtype, device=src.device)
    if src.is_cuda:
        dist.all_gather_into_tensor(out, buf, group=group)
    else:
        dist.all_gather(list(out.view(world, maxlen).unbind(0)), buf, group=group)
    return out.view(world, maxlen).to(t.device)


def gather_column(local, my_rgs, shards, row_counts, group=None):
    """All-gather fixed-width decoded slices into the full column on every rank.

    local:  1-D tensor = this rank's row groups (my_rgs, ascending) decoded back to back.
    shards: every rank's row-group list (shard_row_groups output).
    Returns the concatenated column (rows of all row groups in row-group order).
    """
    counts = np.asarray(row_counts, dtype=np.int64)
    per_rank = [int(counts[s].sum()) for s in shards]
    assert local.numel() == per_rank[dist.get_rank(group)], (local.numel(), per_rank)
    parts = _all_gather_padded(local, max(per_rank) if per_rank else 0, group)
    offs = row_group_offsets(counts)
    full = torch.empty(int(counts.sum()), dtype=local.dtype, device=local.device)
    for r, rgs in enumerate(shards):
        pos = 0
        for rg in rgs:
            n = int(counts[rg])
            full[int(offs[rg]): int(offs[rg]) + n] = parts[r][pos: pos + n]
            pos += n
    return full


def gather_binary(offsets, data, my_rgs, shards, row_counts, group=None):
    """All-gather a BYTE_ARRAY column (int64 offsets[n + 1] from 0 + value bytes) whose rows are this
    rank's row groups back to back. Returns (offsets[N + 1], data) of the full column in row-group
    order: one all-gather of the byte totals (int64 per rank), their exclusive scan, then the offsets
    and the bytes, each row group's offsets rebased onto the concatenated bytes."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = np.asarray(row_counts, dtype=np.int64)
    per_rank = [int(counts[s].sum()) for s in shards]
    n_local = per_rank[rank]
    assert offsets.numel() == n_local + 1, (offsets.numel(), n_local)
    total = offsets[n_local: n_local + 1].to(torch.int64)
    totals = _all_gather_padded(total, 1, group).view(world).cpu().numpy()
    byte_base = np.concatenate([[0], np.cumsum(totals)])
    d_parts = _all_gather_padded(data[: int(totals[rank])], int(totals.max()) if world else 0, group)
    o_parts = _all_gather_padded(offsets[:n_local], max(per_rank), group)
    rg_off = row_group_offsets(counts)
    # bytes of the full column are the ranks' bytes in row-group order; each row group's byte range
    # inside its rank comes from that rank's own offsets
    full_off = torch.empty(int(counts.sum()) + 1, dtype=torch.int64, device=offsets.device)
    segs = []
    rg_src = {}
    for r, rgs in enumerate(shards):
        pos = 0
        for rg in rgs:
            rg_src[rg] = (r, pos)
            pos += int(counts[rg])
    o_host = [o_parts[r, : per_rank[r]].cpu().numpy() for r in range(world)]
    run = 0
    for rg in range(len(counts)):
        r, pos = rg_src[rg]
        n = int(counts[rg])
        lo = int(o_host[r][pos]) if n else 0
        hi = int(o_host[r][pos + n]) if pos + n < per_rank[r] else int(totals[r])
        full_off[int(rg_off[rg]): int(rg_off[rg]) + n] = o_parts[r, pos: pos + n] - lo + run
        segs.append(d_parts[r, lo:hi])
        run += hi - lo
    full_off[-1] = run
    full_data = torch.cat(segs) if segs else torch.zeros(0, dtype=data.dtype, device=data.device)
    assert run == int(byte_base[-1])
    return full_off, full_data
