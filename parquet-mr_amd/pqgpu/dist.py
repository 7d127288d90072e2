"""Row-group sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

A row group's column chunks decode with no cross-chunk state, so
ranks decode disjoint row groups with no data-path collective. The only exchange
is optional: concatenating the decoded slices into one full column on every
rank (all-gather over RCCL). Output offsets of each row group are prefix sums
of footer row counts, so no offsets need exchanging for fixed-width columns.
Reference parallelism being restated: Hadoop InputSplits at row-group
granularity (ParquetInputFormat.getSplits :350, generateSplits :786).
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


def gather_column(local, my_rgs, shards, row_counts, group=None):
    """All-gather fixed-width decoded slices into the full column on every rank.

    local:  1-D tensor = this rank's row groups (my_rgs, ascending) decoded back to back.
    shards: every rank's row-group list (shard_row_groups output).
    Returns the concatenated column (rows of all row groups in row-group order).
    """
    world = dist.get_world_size(group)
    counts = np.asarray(row_counts, dtype=np.int64)
    per_rank = [int(counts[s].sum()) for s in shards]
    maxlen = max(per_rank) if per_rank else 0
    buf = torch.zeros(maxlen, dtype=local.dtype, device=local.device)
    buf[: local.numel()] = local
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    offs = row_group_offsets(counts)
    full = torch.empty(int(counts.sum()), dtype=local.dtype, device=local.device)
    for r, rgs in enumerate(shards):
        pos = 0
        for rg in rgs:
            n = int(counts[rg])
            full[int(offs[rg]): int(offs[rg]) + n] = parts[r][pos: pos + n]
            pos += n
    return full
