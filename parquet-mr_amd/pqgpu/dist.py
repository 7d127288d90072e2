"""Row-group sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

A row group's column chunks decode with no cross-chunk state, so ranks decode
disjoint row groups with no data-path collective. The only exchange is the final column
concatenation, when a consumer wants the full column on every rank:

  * shards are contiguous runs of row groups in file order, balanced by encoded bytes (the
    Hadoop split: ParquetInputFormat.generateSplitInfo assigns row groups to splits in file order
    by compressed size, parquet-hadoop/src/main/java/org/apache/parquet/hadoop/ParquetInputFormat.java
    :807-841, via getSplits :350 / generateSplits :786), so the full column is the ranks' slices
    back to back: rank r's rows land at a fixed offset of the output;
  * fixed-width columns: one all-gather straight into the output (`all_gather_into_tensor` when
    the slices are equal, otherwise one batch of point-to-point copies, each rank's slice sent once
    to every peer: on xGMI's fully connected links the peers are direct neighbours), no padding;
  * BYTE_ARRAY columns: one all-gather of every rank's byte total (one int64 each), their exclusive
    scan gives every rank's byte base, each rank rebases its own offsets on the device (one add), and
    the rebased offsets and the value bytes are gathered into the output the same way. No O(rows)
    host transfer and no per-row-group host loop.
"""
import numpy as np
import torch
import torch.distributed as dist


def shard_row_groups(sizes, world):
    """Contiguous row-group ranges, one per rank, balanced by encoded bytes: rank r takes the row
    groups whose byte midpoint falls in [r, r + 1) * total / world (file order kept, as Hadoop's
    splits keep it). Returns, per rank, its ascending list of row-group indices."""
    sizes = np.asarray(sizes, dtype=np.float64)
    out = [[] for _ in range(world)]
    if sizes.size == 0:
        return out
    total = float(sizes.sum())
    mid = np.cumsum(sizes) - sizes / 2
    if total > 0:
        owner = np.minimum((mid * world / total).astype(np.int64), world - 1)
    else:
        owner = np.arange(sizes.size) * world // sizes.size
    for i, r in enumerate(owner):
        out[int(r)].append(i)
    return out


def row_group_offsets(row_counts):
    """First output row of each row group in the concatenated column."""
    return np.concatenate([[0], np.cumsum(np.asarray(row_counts, dtype=np.int64))])[:-1]


def _check_contiguous(shards):
    flat = [g for s in shards for g in s]
    assert flat == list(range(len(flat))), "shards must be contiguous row-group ranges in rank order"


def _on_backend(t, group):
    """gloo collectives run on host tensors; RCCL (backend "nccl") on device tensors."""
    return t.cpu() if dist.get_backend(group) == "gloo" else t


def all_gather_into(out, local, sizes, group=None):
    """All-gather 1-D slices of per-rank `sizes` (elements) into `out` = the slices back to back in
    rank order, with no padding: all_gather_into_tensor when every size is equal, otherwise one
    batch of point-to-point sends / receives (rank r's slice to every peer)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    assert local.numel() == sizes[rank] and out.numel() == sum(sizes)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    dst = _on_backend(out, group)
    src = _on_backend(local, group)
    if world == 1 or len(set(sizes)) == 1:
        if world == 1:
            dst.copy_(src)
        elif dst.is_cuda:
            dist.all_gather_into_tensor(dst, src.contiguous(), group=group)
        else:
            dist.all_gather(list(dst.view(world, sizes[0]).unbind(0)), src.contiguous(), group=group)
    else:
        dst[int(off[rank]): int(off[rank + 1])].copy_(src)
        ops = []
        for peer in range(world):
            if peer == rank:
                continue
            if sizes[rank]:
                ops.append(dist.P2POp(dist.isend, src.contiguous(), dist.get_global_rank(group, peer)
                                      if group is not None else peer, group))
            if sizes[peer]:
                ops.append(dist.P2POp(dist.irecv, dst[int(off[peer]): int(off[peer + 1])],
                                      dist.get_global_rank(group, peer) if group is not None else peer, group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
    if dst is not out:
        out.copy_(dst)
    return out


def gather_column(local, my_rgs, shards, row_counts, group=None):
    """All-gather fixed-width decoded slices into the full column on every rank.

    local:  1-D tensor = this rank's row groups (my_rgs, ascending) decoded back to back.
    shards: every rank's contiguous row-group range (shard_row_groups output).
    Returns the concatenated column (rows of all row groups in row-group order).
    """
    _check_contiguous(shards)
    counts = np.asarray(row_counts, dtype=np.int64)
    per_rank = [int(counts[s].sum()) for s in shards]
    full = torch.empty(int(counts.sum()), dtype=local.dtype, device=local.device)
    return all_gather_into(full, local, per_rank, group)


def gather_binary(offsets, data, my_rgs, shards, row_counts, group=None):
    """All-gather a BYTE_ARRAY column (int64 offsets[n + 1] from 0 + value bytes) whose rows are this
    rank's row groups back to back. Returns (offsets[N + 1], data) of the full column in row-group
    order: one all-gather of the byte totals (one int64 per rank); every rank adds its byte base to
    its own offsets on the device; the rebased offsets and the bytes are gathered into the outputs."""
    _check_contiguous(shards)
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = np.asarray(row_counts, dtype=np.int64)
    per_rank = [int(counts[s].sum()) for s in shards]
    n_local = per_rank[rank]
    assert offsets.numel() == n_local + 1, (offsets.numel(), n_local)
    total = offsets[n_local: n_local + 1].to(torch.int64)
    totals_t = torch.empty(world, dtype=torch.int64, device=offsets.device)
    all_gather_into(totals_t, total, [1] * world, group)
    totals = [int(x) for x in totals_t.cpu().tolist()]        # world int64s
    base = int(np.sum(totals[:rank], dtype=np.int64))
    rebased = offsets[:n_local] + base                       # device rebase onto the full byte buffer
    full_off = torch.empty(int(counts.sum()) + 1, dtype=torch.int64, device=offsets.device)
    all_gather_into(full_off[:-1], rebased, per_rank, group)
    full_off[-1] = int(np.sum(totals, dtype=np.int64))
    full_data = torch.empty(int(np.sum(totals, dtype=np.int64)), dtype=data.dtype, device=data.device)
    all_gather_into(full_data, data[: totals[rank]], totals, group)
    return full_off, full_data
