#!/usr/bin/env python3
"""Benchmark: decoded values/s + GiB/s on device-resident int64 RLE_DICTIONARY pages
(BASELINE.json configs[1]: 100M rows, 1k-cardinality dictionary, Zipf(1.5) run
lengths truncated to [1, 4096], parquet-mr V1 pages of 20,000 values, uncompressed).

A step = one decode of the whole 100M-value column chunk (5,000 pages) already
resident in HBM, into a dense int64 column in HBM. With --gpus N (torch.distributed
launcher) every rank decodes its own 100M-row row group (row groups shard
one-per-GPU, no data-path collective: weak scaling); value = all ranks' values /
max-over-ranks time.

Prints ONE JSON line on rank 0. Extra objects: "roofline" (dominant kernel
k_dict<8>, HBM-bound), "cpu_baseline" (the oracle's value-at-a-time port of
the reference reader, 1 thread, bounded sample) and, at N=1, "e2e_host_path" (the
PCIe-inclusive pqg_decode_host rate with the pinned D2H link ceiling measured in the
same run; never `value`).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(REPO, "parquet-mr_amd"), os.path.join(REPO, "tools")]

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md: 8.0 TB/s spec)
DOMINANT_KERNEL = "void pqg::k_dict_fused<8>"
TRAFFIC_JSON = os.path.join(REPO, "profiles", "traffic_latest.json")


def workload_key(rows, zipf):
    return f"C2 rows={rows} zipf={zipf}"


def make_c2(n_rows, seed_dict=42, seed_runs=43, a=1.5, card=1000, max_run=4096, page_rows=20000):
    """Config 2 input: the dictionary column as parquet-mr would write it (tools/workloads.py)."""
    import workloads
    return workloads.make_c2(n_rows, seed_dict, seed_runs, a, card, max_run, page_rows)


def cpu_baseline(batch, n_values, budget_s):
    """The oracle (value-at-a-time C port of RunLengthBitPackingHybridDecoder.readInt ->
    Dictionary.decodeToLong, 1 thread) on the same pages, repeated for ~budget_s."""
    sys.path.insert(0, REPO)
    from oracle import pqref
    t0 = time.perf_counter()
    reps = 0
    while True:
        r = pqref.decode_batch(batch)
        assert r.code == 0
        reps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": reps * n_values / dt, "unit": "values/s", "cores": 1, "kind": "port",
            "sample": f"{reps} x full {n_values / 1e6:.0f}M-value chunk ({batch.n_pages} pages), "
                      f"{dt:.1f} s, oracle/pqref.c -O3, single thread"}


def cpu_baseline_mt(chunk, n_values, threads, budget_s):
    """The same oracle on `threads` host threads, pages split into contiguous groups (pages of a
    required dictionary column are independent once the dictionary is read; ctypes releases the
    GIL during the C decode)."""
    from concurrent.futures import ThreadPoolExecutor
    from tools.synth import writer
    sys.path.insert(0, REPO)
    from oracle import pqref
    groups = np.array_split(np.arange(len(chunk.pages)), threads)
    subs = []
    for g in groups:
        c = writer.ColumnChunk(physical_type=chunk.physical_type, dict_page=chunk.dict_page,
                               dict_num_values=chunk.dict_num_values, dict_encoding=chunk.dict_encoding)
        c.pages = [chunk.pages[i] for i in g]
        subs.append(writer.build_batch([c]))
    with ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        reps = 0
        while True:
            for r in ex.map(pqref.decode_batch, subs):
                assert r.code == 0
            reps += 1
            if time.perf_counter() - t0 >= budget_s:
                break
        dt = time.perf_counter() - t0
    return {"value": reps * n_values / dt, "unit": "values/s", "cores": threads, "kind": "port",
            "sample": f"{reps} x full chunk, {threads} threads over page groups, {dt:.1f} s"}


def pyarrow_baseline(values, budget_s, threads):
    """Third-party reference point (not the reference): Arrow C++ (pyarrow) reading the same
    values written by pyarrow as one dictionary-encoded int64 column, uncompressed, V1 pages."""
    try:
        import pyarrow as pa
        import pyarrow.parquet as pq
    except Exception as e:  # pyarrow absent on the host
        return {"unavailable": str(e)}
    sink = pa.BufferOutputStream()
    pq.write_table(pa.table({"c2": pa.array(values)}), sink, compression="NONE", use_dictionary=True,
                   data_page_version="1.0", row_group_size=len(values))
    buf = sink.getvalue()
    pa.set_cpu_count(threads)
    t0 = time.perf_counter()
    reps = 0
    while True:
        t = pq.read_table(pa.BufferReader(buf), use_threads=True)
        reps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": reps * len(values) / dt, "unit": "values/s", "cores": threads, "kind": "third-party",
            "sample": f"pyarrow {pa.__version__} read_table of the same 100M values (its own pages), {reps} reps"}


def store_ceiling(nbytes, device, stream, reps=10):
    """Write-only HBM rate of this box for the headline's output size, in GB/s: torch's fill_ of an
    nbytes int64 buffer on the decode stream (the expansion's stores alone, without its reads or walks),
    best of `reps`, timed with HIP events on that stream. The decode's achieved rate is reported against
    both this and the nominal 8 TB/s."""
    import torch
    buf = torch.empty(nbytes // 8, dtype=torch.int64, device=device)
    best = None
    with torch.cuda.stream(stream):
        buf.fill_(0)
        for r in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            buf.fill_(r)
            e1.record(stream)
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None or ms < best else best
    del buf
    return nbytes / (best / 1e3) / 1e9


def link_ceiling(out_bytes, in_bytes, device, reps=5):
    """The PCIe link alone on this box, best of `reps`, in GB/s: one pinned hipMemcpyAsync of the
    decoded column's size (device -> host) and of the encoded pages' size (host -> device); the
    decoded size as 32 MiB pieces alternating over two streams (two DMA engines, as pqg_decode_host
    issues it); and the host's own copy of that size from pinned into a touched pageable array
    (torch's threaded CPU copy), the last stage of pqg_decode_host."""
    import torch
    res = {}
    s = torch.cuda.Stream(device)
    s2 = torch.cuda.Stream(device)

    def best_of(fn, sync):
        best = None
        for _ in range(reps):
            torch.cuda.synchronize(device)
            t0 = time.perf_counter()
            fn()
            sync()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return best

    for name, n, d2h in (("d2h_pinned_gbs", out_bytes, True), ("h2d_pinned_gbs", in_bytes, False)):
        dev_t = torch.empty(n, dtype=torch.uint8, device=device)
        host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        host.fill_(1)

        def one():
            with torch.cuda.stream(s):
                (host.copy_(dev_t, non_blocking=True) if d2h else dev_t.copy_(host, non_blocking=True))
        res[name] = n / best_of(one, s.synchronize) / 1e9
        if d2h:
            piece = 32 << 20

            def two():
                for k, a in enumerate(range(0, n, piece)):
                    with torch.cuda.stream(s2 if k & 1 else s):
                        host[a:a + piece].copy_(dev_t[a:a + piece], non_blocking=True)
            res["d2h_pinned_2streams_gbs"] = n / best_of(two, lambda: (s.synchronize(), s2.synchronize())) / 1e9
            page = torch.empty(n, dtype=torch.uint8)
            page.fill_(0)
            res["host_pinned_to_pageable_gbs"] = n / best_of(lambda: page.copy_(host), lambda: None) / 1e9
            res["host_copy_threads"] = torch.get_num_threads()
            del page
        del dev_t, host
    res["bytes"] = {"d2h": out_bytes, "h2d": in_bytes}
    return res


def launch_ranks(n):
    """`--gpus N` run without a launcher: start N ranks under torch.distributed.run (one process per
    GPU, rendezvous on 127.0.0.1) as a CHILD process and exit with its code. Nothing here touches
    the GPU, so no process that initialised HIP is replaced."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, PQG_BENCH_LAUNCHED="1")
    return subprocess.call(cmd, env=env)


def init_ranks(args):
    """-> (world, rank, local_rank, device index). World size is what the process group reports."""
    import torch
    import torch.distributed as dist
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world_env != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world_env} ranks; reporting {world_env}",
              file=sys.stderr)
    ndev = torch.cuda.device_count()
    dev = local % max(ndev, 1)
    torch.cuda.set_device(dev)
    world = 1
    if world_env > 1:
        backend = args.backend or ("nccl" if ndev >= world_env else "gloo")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:  # fewer GPUs than ranks (rehearsal on a 1-GPU box): ranks share the GPU, gloo collectives
            dist.init_process_group("gloo")
        world = dist.get_world_size()
        rank = dist.get_rank()
    return world, rank, local, dev


def step_time(gpu_s, wall_s):
    """-> (seconds of the timed launches, timer): the HIP event interval on the decoder's stream (max over
    ranks), unless it exceeds the host wall clock around the same launches (max over ranks), which it
    cannot do when both are right (seen with two ranks sharing one GPU: a 100 s event interval inside a
    2-minute job); the wall clock, which also holds the barrier and launch overhead, is then reported."""
    if gpu_s <= wall_s * 1.02:
        return gpu_s, "hip events"
    return wall_s, "host wall clock (the HIP event interval exceeded it)"


def run_c4(args, world, rank, devi):
    """C4 (BASELINE configs[3]): TPC-H lineitem-shaped 16 columns, `--rows` rows in total (default 1 B)
    in row groups of 1M rows, sharded over the ranks by encoded bytes (dist.shard_row_groups, the
    Hadoop row-group split); strong scaling. A step = one plan launch decoding every page of the
    rank's row groups (16 columns: DELTA int64 keys / int32 dates, PLAIN doubles, dictionary int32
    and strings, PLAIN comment strings) into the rank's slice of each column. The inputs are
    `--c4-templates` distinct synthetic row groups laid out repeatedly (row group g = template
    g mod T): every copy's pages are decoded, none is skipped or cached."""
    import torch
    import torch.distributed as dist
    import lineitem as LI
    from pqgpu import abi, decoder as D, dist as pdist
    from tools.synth import writer

    t_gen = time.perf_counter()
    keep = [int(k) for k in args.c4_cols.split(",")] if args.c4_cols else None
    shard = LI.Shard(args.rows, world, rank, args.c4_templates, keep=keep)
    n_keep = len(shard.keep)
    rg_rows, n_rg, T, templates, shards, mine = shard.rg_rows, shard.n_rg, shard.T, shard.templates, shard.shards, shard.mine
    batch, col_of = shard.batch, shard.col_of
    t_gen = time.perf_counter() - t_gen
    enc_bytes = int(batch.pages["size"].sum()) + sum(int(c["dict_size"]) for c in batch.columns if c["dict_offset"] >= 0)

    dec = D.Decoder(devi, poison=0xA5)
    if args.dict_split:
        dec.set_dispatch(abi.DISPATCH_DICT_FUSED, 0)
    _ab_dispatch(dec)
    if args.plain_mode is not None:
        dec.set_dispatch(abi.DISPATCH_PLAIN_ONE_PASS, args.plain_mode)
    dbatch = dec.upload(batch)
    cols, st = dec.decode(dbatch)  # sizes the BYTE_ARRAY buffers
    for c in cols:  # poison: the plan's first launch must write every element itself
        for t in (c.values, c.def_levels, c.rep_levels, c.binary_data):
            if t is not None:
                t.fill_(0xA5)
    plan = dec.plan(dbatch, cols)

    def verify(what):
        shard.verify(cols, dec.device, what)

    plan.launch()  # first launch of the fresh plan, checked
    rc, st = plan.sync()
    assert rc == 0, st.message
    if not args.no_verify:
        verify("first launch")
    for _ in range(args.warmup):
        plan.launch()
    rc, st = plan.sync()
    assert rc == 0, st.message
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record(dec.stream)
    for k in range(args.steps):
        plan.launch()
        ev[k + 1].record(dec.stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    rc, st = plan.sync()
    assert rc == 0, st.message
    if not args.no_verify:
        verify("after the timed launches")
    per_launch_ms = [ev[k].elapsed_time(ev[k + 1]) for k in range(args.steps)]
    gpu_s = sum(per_launch_ms) / 1e3
    if world > 1:
        print(json.dumps({"rank": rank, "launch_ms": [round(x, 4) for x in per_launch_ms],
                          "plan_reruns": {"timeout": plan.timeout_fallbacks, "plain": plan.plain_fallbacks}}),
              file=sys.stderr, flush=True)
    out_bytes = 0
    for i, cd in enumerate(batch.columns):
        n = cols[i].n_values
        out_bytes += 8 * (n + 1) + int(cols[i].offsets()[-1].item()) if cd["physical_type"] == abi.BYTE_ARRAY \
            else n * abi.elem_width(cd["physical_type"], cd["type_length"])
    t = torch.tensor([gpu_s, wall, float(len(mine) * rg_rows), float(enc_bytes + out_bytes)], dtype=torch.float64)
    rows_all = torch.tensor([float(len(mine) * rg_rows), float(enc_bytes + out_bytes)], dtype=torch.float64)
    if world > 1:
        dev = f"cuda:{devi}" if dist.get_backend() == "nccl" else "cpu"
        t, rows_all = t.to(dev), rows_all.to(dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(rows_all)
    t_max, timer = step_time(float(t[0].item()), float(t[1].item()))
    total_rows, total_bytes = float(rows_all[0].item()), float(rows_all[1].item())

    gather = None
    if world > 1 and not args.no_gather:
        # final concatenation of two representative columns over RCCL: l_orderkey (int64, fixed width)
        # and l_comment (BYTE_ARRAY: byte-total all-gather + offset rebase), timed separately
        counts = [rg_rows] * n_rg
        ok_col, cm_col = cols[col_of[(0, -1)]], cols[col_of[(15, -1)]]
        res = {}
        for name, fn in (("l_orderkey", lambda: pdist.gather_column(ok_col.typed(), mine, shards, counts)),
                         ("l_comment", lambda: pdist.gather_binary(cm_col.offsets(), cm_col.binary_data, mine, shards,
                                                                  counts))):
            fn()
            dist.barrier()
            torch.cuda.synchronize()
            tg = time.perf_counter()
            r = fn()
            torch.cuda.synchronize()
            dist.barrier()
            nbytes = r.numel() * r.element_size() if not isinstance(r, tuple) else sum(x.numel() * x.element_size() for x in r)
            gs = torch.tensor([time.perf_counter() - tg], dtype=torch.float64)
            gs = gs.to(f"cuda:{devi}") if dist.get_backend() == "nccl" else gs
            dist.all_reduce(gs, op=dist.ReduceOp.MAX)
            res[name] = {"full_column_bytes": nbytes, "seconds": float(gs.item()),
                         "gb_per_s": nbytes / float(gs.item()) / 1e9}
            del r
        gather = {"collective": f"all_gather ({dist.get_backend()})", "columns": res,
                  "note": "timed separately; not part of value (decode-only rate)"}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, REPO)
        from oracle import pqref
        b1 = writer.build_batch([templates[0][0][k] for k in shard.keep])
        t1, reps = time.perf_counter(), 0
        while True:
            r = pqref.decode_batch(b1)
            assert r.code == 0
            reps += 1
            if time.perf_counter() - t1 >= args.cpu_budget:
                break
        dt = time.perf_counter() - t1
        cpu = {"value": reps * rg_rows * n_keep / dt, "unit": "values/s", "cores": 1, "kind": "port",
               "sample": f"{reps} x one 1M-row, {n_keep}-column row group, oracle/pqref.c single thread, {dt:.1f} s"}
    if rank == 0:
        value = total_rows * n_keep * args.steps / t_max
        # HBM traffic of one launch (every kernel's PMC FETCH_SIZE x 2 + WRITE_SIZE per dispatch, summed;
        # tools/c4_traffic.sh) when it was measured on this workload
        c4_traffic, c4_traffic_bytes, c4_traffic_src = None, None, None
        tj_path = os.path.join(REPO, "profiles", "traffic_c4_latest.json")
        if os.path.exists(tj_path) and world == 1:
            tj = json.load(open(tj_path))
            if tj.get("rows") == int(total_rows) and tj.get("columns") == list(shard.keep):
                c4_traffic_bytes = tj["traffic_bytes_per_launch"]
                c4_traffic = c4_traffic_bytes / (t_max / args.steps) / 1e9
                c4_traffic_src = os.path.relpath(tj_path, REPO)
        out = {
            "metric": "decoded values/s, device-resident C4 lineitem 16 columns",
            "value": value, "unit": "values/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": t_max * 1e3 / args.steps, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "mixed (int32/int64/f64/bytes)", "data": "synthetic",
            "config": {"workload": "C4: TPC-H lineitem-shaped 16 required columns (DELTA int64 keys / int32 dates, "
                                   "PLAIN doubles, RLE_DICTIONARY int32 + strings, PLAIN comment), parquet-mr V1 "
                                   "pages of 20,000 values, uncompressed, 1M-row row groups sharded over ranks",
                       "rows_total": int(total_rows), "row_groups_total": n_rg, "row_groups_this_rank": len(mine),
                       "distinct_row_groups": T, "pages_this_rank": batch.n_pages,
                       "pqg_columns_this_rank": len(batch.columns), "parallelism": f"row-group shard x{world}",
                       "lineitem_columns": shard.keep},
            "gb_per_s": total_bytes * args.steps / t_max / 1e9,
            "hbm_frac_per_gpu": total_bytes * args.steps / t_max / 1e9 / world / HBM_PEAK_GBS,
            "kernels_per_launch": plan.kernel_count,
            # the bound of the whole launch (13 kernels, each HBM-bound integer / byte work): algorithmic
            # bytes = every column's encoded page bytes read + dense outputs written, per GPU
            "roofline": {"bound": "hbm", "achieved": total_bytes / world / (t_max / args.steps) / 1e9,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": total_bytes / world / (t_max / args.steps) / 1e9 / HBM_PEAK_GBS,
                         "traffic": c4_traffic, "traffic_bytes_per_launch": c4_traffic_bytes,
                         "traffic_source": c4_traffic_src,
                         "kernel": "whole plan launch (all kernels of the shard)",
                         "algorithmic_bytes_per_launch": total_bytes / world},
            "verified": None if args.no_verify else "every row group x column slice == its generated values, first launch "
                                                    "of a fresh plan and after the timed launches",
            "cpu_baseline": cpu, "input_gen_s": t_gen,
            "timer": timer, "wall_ms_per_step": float(t[1].item()) * 1e3 / args.steps,
            "rank0_launch_ms": [round(x, 4) for x in per_launch_ms],
            "rank0_plan_reruns": {"timeout": plan.timeout_fallbacks, "plain": plan.plain_fallbacks,
                                  "null_hint": plan.null_hint_fallbacks},
        }
        if gather:
            out["gather"] = gather
        print(json.dumps(out), flush=True)
    plan.close()
    dec.close()
    if world > 1:
        dist.destroy_process_group()


def _ab_dispatch(dec):
    """A/B runs only: PQGPU_DISPATCH="key=value,..." (abi.DISPATCH_* keys) overrides the measured defaults."""
    for kv in filter(None, os.environ.get("PQGPU_DISPATCH", "").split(",")):
        k, v = kv.split("=")
        dec.set_dispatch(int(k), int(v))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["c2", "c4"], default="c2",
                    help="c2: the headline (BASELINE metric); c4: lineitem 16 columns, strong scaling")
    ap.add_argument("--rows", type=int, default=None, help="c2: rows per GPU (100M); c4: rows in total (1B)")
    ap.add_argument("--c4-templates", type=int, default=4, help="c4: distinct synthetic row groups")
    ap.add_argument("--plain-mode", type=int, default=None,
                    help="PQG_DISPATCH_PLAIN_ONE_PASS override (A/B of the PLAIN BYTE_ARRAY kernels)")
    ap.add_argument("--dict-split", action="store_true",
                    help="diagnostics: dictionary walk and expansion as two launches (PQG_DISPATCH_DICT_FUSED = 0)")
    ap.add_argument("--c4-cols", default=None,
                    help="c4 diagnostics: comma-separated lineitem columns to decode (default: all 16)")
    ap.add_argument("--zipf", type=float, default=1.5)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-gather", action="store_true", help="N > 1: skip the timed RCCL all-gather of the column")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default=None)
    ap.add_argument("--e2e", action="store_true",
                    help="time the host-bytes-in / host-array-out path (default on at N=1, rank 0)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host path (profiling runs)")
    ap.add_argument("--traffic-json", default=TRAFFIC_JSON,
                    help="rocprofv3 PMC traffic summary of this kernel (tools/pmc_summary.py --json)")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    import torch
    import torch.distributed as dist
    from pqgpu import decoder as D
    from tools.synth import writer

    world, rank, local, devi = init_ranks(args)
    if args.workload == "c4":
        args.rows = args.rows or 1_000_000_000
        return run_c4(args, world, rank, devi)
    args.rows = args.rows or 100_000_000

    t_gen = time.perf_counter()
    # each rank owns one row group: same dictionary seed, its own run stream
    chunk, dict_vals, ids = make_c2(args.rows, seed_runs=43 + 1000 * rank, a=args.zipf)
    batch = writer.build_batch([chunk])
    t_gen = time.perf_counter() - t_gen
    data_bytes = int(sum(len(p.body) for p in chunk.pages))

    dec = D.Decoder(devi, poison=0xA5)
    if args.dict_split:
        from pqgpu import abi
        dec.set_dispatch(abi.DISPATCH_DICT_FUSED, 0)
    _ab_dispatch(dec)
    dbatch = dec.upload(batch)
    cols = dec.alloc_columns(batch)  # poisoned: an element no launch writes cannot pass the check
    plan = dec.plan(dbatch, cols)
    stream = dec.stream
    exp = None
    if not args.no_verify:
        exp = torch.from_numpy(dict_vals[ids]).to(dec.device)
        plan.launch()  # the FIRST launch of a fresh plan is checked (not one after warm-up rewrites)
        rc, st = plan.sync()
        assert rc == 0, st.message
        assert torch.equal(cols[0].typed(), exp), "first launch: decoded column differs from the generated values"
    for _ in range(args.warmup):
        plan.launch()
    rc, st = plan.sync()
    assert rc == 0, st.message

    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record(stream)
    for k in range(args.steps):
        plan.launch()
        ev[k + 1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    rc, st = plan.sync()
    assert rc == 0, st.message
    if exp is not None:
        assert torch.equal(cols[0].typed(), exp), "after the timed launches: decoded column differs"
    per_launch_ms = [ev[k].elapsed_time(ev[k + 1]) for k in range(args.steps)]
    gpu_ms = sum(per_launch_ms)
    t = torch.tensor([gpu_ms / 1e3, wall], dtype=torch.float64)
    if world > 1:
        t = t.to(f"cuda:{devi}") if dist.get_backend() == "nccl" else t
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max, timer = step_time(float(t[0].item()), float(t[1].item()))

    gather = None
    if world > 1 and not args.no_gather:
        # the final column concatenation (north_star: RCCL/xGMI gather only for it), timed on its own:
        # every rank ends with the full world x rows column; checked by a checksum of checksums
        from pqgpu import dist as pdist
        shards = [[r] for r in range(world)]
        counts = [args.rows] * world
        local_col = cols[0].typed()
        full = pdist.gather_column(local_col, [rank], shards, counts)  # warm-up (communicator setup)
        del full
        dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        full = pdist.gather_column(local_col, [rank], shards, counts)
        torch.cuda.synchronize()
        dist.barrier()
        g_s = torch.tensor([time.perf_counter() - tg], dtype=torch.float64)
        csum = torch.tensor([int(local_col.sum().item()) & (2**63 - 1)], dtype=torch.int64)
        g_s = g_s.to(f"cuda:{devi}") if dist.get_backend() == "nccl" else g_s
        csum = csum.to(g_s.device)
        dist.all_reduce(g_s, op=dist.ReduceOp.MAX)
        dist.all_reduce(csum)
        ok = (int(full.sum().item()) & (2**63 - 1)) == (int(csum.item()) & (2**63 - 1)) and full.numel() == world * args.rows
        g = float(g_s.item())
        recv = (world - 1) * args.rows * 8
        gather = {"collective": f"all_gather ({dist.get_backend()})", "bytes_received_per_rank": recv,
                  "seconds": g, "gb_per_s_per_rank": recv / g / 1e9, "checksum_ok": bool(ok),
                  "note": "timed separately; not part of value (decode-only rate)"}
        del full

    n = args.rows
    total_values = n * world * args.steps
    value = total_values / t_max
    ms_per_step = t_max * 1e3 / args.steps
    avg_launch_s = float(np.mean(per_launch_ms)) / 1e3
    algo_bytes = n * 8 + data_bytes  # per launch: int64 out + encoded data-page bytes read
    achieved = algo_bytes / avg_launch_s / 1e9
    st_ceil = store_ceiling(n * 8, cols[0].typed().device, stream)

    e2e = None
    if rank == 0 and (args.e2e or (world == 1 and not args.no_e2e)):
        times, native_s = [], []
        for _ in range(3):  # best of 3 (the first call also allocates and pins the staging buffers)
            t1 = time.perf_counter()
            rc2, st2, res, _ = dec.decode_host(batch, prefault=True)
            times.append(time.perf_counter() - t1)
            native_s.append(dec.last_native_s)
            assert rc2 == 0
        e2e_s = min(native_s)
        staged_s = []
        for _ in range(3):  # the staged path: outputs stay in the library's pinned buffer (no host copy)
            rc3, _, res3, _ = dec.decode_staged(batch)
            staged_s.append(dec.last_native_s)
            assert rc3 == 0 and res3[0]["n_values"] == n
        link = link_ceiling(n * 8, data_bytes, dec.device)
        # the link's share of the host path: the output's D2H at the measured pinned ceilings
        d2h_floor_s = n * 8 / (link["d2h_pinned_gbs"] * 1e9)
        d2h2_floor_s = n * 8 / (link["d2h_pinned_2streams_gbs"] * 1e9)
        e2e = {"values_per_s": n / e2e_s, "seconds": e2e_s, "native_call_s": native_s,
               "output_gb_per_s": n * 8 / e2e_s / 1e9, "link": link,
               "frac_of_d2h_ceiling": d2h_floor_s / e2e_s,
               "frac_of_d2h_2streams_ceiling": d2h2_floor_s / e2e_s,
               "with_python_alloc_s": times,
               "path": "pqg_decode_host (one C call: host page bytes -> pinned -> H2D, plan, decode, sync, "
                       "chunked D2H -> caller's int64 array); output array allocated and touched beforehand",
               "staged": {"seconds": min(staged_s), "native_call_s": staged_s,
                          "output_gb_per_s": n * 8 / min(staged_s) / 1e9,
                          "frac_of_d2h_2streams_ceiling": d2h2_floor_s / min(staged_s),
                          "path": "pqg_decode_staged (page bytes already in the pinned input; outputs left in "
                                  "the pinned output for the caller to read in place)"}}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(batch, n, args.cpu_budget)
        threads = min(16, os.cpu_count() or 1)  # the GPU box's CPU share is 16 cores
        cpu["multi_thread"] = cpu_baseline_mt(chunk, n, threads, args.cpu_budget / 2)
        cpu["pyarrow"] = pyarrow_baseline(dict_vals[ids], args.cpu_budget / 2, threads)

    traffic, traffic_bytes, traffic_src = None, None, None
    if os.path.exists(args.traffic_json):
        # HBM bytes per launch of the same kernel from the committed rocprofv3 --pmc passes
        # (tools/pmc_summary.py: FETCH_SIZE x2 + WRITE_SIZE, gfx950 corrections); reported in the
        # unit of `achieved` (bytes per launch / this run's average launch time)
        tj = json.load(open(args.traffic_json))
        v = tj.get("kernels", {}).get(DOMINANT_KERNEL)
        if v and tj.get("workload") == workload_key(n, args.zipf):
            traffic_bytes = v["traffic_bytes"]
            traffic = traffic_bytes / avg_launch_s / 1e9
            traffic_src = os.path.relpath(args.traffic_json, REPO)

    if rank == 0:
        out = {
            "metric": "decoded values/s, device-resident int64 RLE_DICTIONARY pages",
            "value": value,
            "unit": "values/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic",
            "config": {"workload": "C2: int64 RLE_DICTIONARY, 1k-cardinality dictionary (w=10), "
                                   f"Zipf(a={args.zipf}) run lengths in [1,4096], parquet-mr V1 pages of 20,000 values, "
                                   "uncompressed, one 100M-row row group per GPU",
                       "rows_per_gpu": n, "pages_per_gpu": batch.n_pages, "encoded_data_bytes_per_gpu": data_bytes,
                       "parallelism": f"row-group shard x{world}"},
            "gib_per_s": value * 8 / 2**30,
            "verified": "first launch of a fresh plan and the state after the timed launches == generated values"
                        if exp is not None else None,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_bytes_per_launch": traffic_bytes, "traffic_source": traffic_src,
                         "kernel": "pqg::k_dict_fused<8> (avg_launch_ms: whole plan launch, one dispatch, incl. the ~6 us dispatch-to-dispatch gap)", "algorithmic_bytes_per_launch": algo_bytes,
                         "avg_launch_ms": avg_launch_s * 1e3,
                         "store_ceiling": st_ceil, "frac_of_store_ceiling": achieved / st_ceil,
                         "store_ceiling_note": "GB/s of a torch fill_ of the 800 MB output on the same stream, "
                                               "best of 10 (write-only; measured live in this run)"},
            "cpu_baseline": cpu,
            "input_gen_s": t_gen,
            "timer": timer, "wall_ms_per_step": float(t[1].item()) * 1e3 / args.steps,
        }
        if gather:
            out["gather"] = gather
        if e2e:
            out["e2e_host_path"] = e2e
        print(json.dumps(out), flush=True)
    plan.close()
    dec.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
