#!/usr/bin/env python3
"""Decode throughput of every BASELINE.json config and encoding family beside the headline.

bench.py prints the ONE headline line (C2). This suite times the other configs and the widened
§8 rows on one GPU, inputs resident in HBM, one JSON line per workload:

  c1_plain_i32   C1: 1M int32 PLAIN, required (plus the host-buffers-in / arrays-out path)
  c2_zipf2       C2 stress variant: Zipf(2.0) run lengths (26 % of ids in bit-packed runs)
  c3_mixed       C3: 8 optional columns (2 int32 + 2 int64 DELTA_BINARY_PACKED, 2 double PLAIN,
                 2 BYTE_ARRAY PLAIN of 4-32 bytes), 10 % nulls, RLE def levels, V2 pages
  c5_levels      C5: LIST<int64> records (Poisson(3) lengths, 10 % null lists / elements),
                 rep + def levels and values, then record assembly (pqg_assemble_schema: list
                 validity + offsets, element validity) in every timed step
  str_plain / str_dict / str_dlba / str_dba   BYTE_ARRAY encodings, 4-32 byte strings
  str_dict_opt   str_dict with 10 % nulls (V1 pages: levels first)
  str_dict_16k   str_dict with a 16,384-entry dictionary (past the LDS-staged dictionary-direct path)
  plain_f64      PLAIN doubles (required)
  bss_f64        BYTE_STREAM_SPLIT doubles
  delta_i64      DELTA_BINARY_PACKED int64 random walk
  delta_i32      DELTA_BINARY_PACKED int32 random walk
  delta_i64_2048 the same values with 2048-value blocks of 8 miniblocks (DuckDB's writer; the block-by-block path)
  (on request) c2_snappy / c2_zstd / c2_lz4 / c2_gzip and plain_i64_{snappy,zstd,lz4,gzip}: the headline
                 pages or an int64 random walk compressed with each codec (decompression timed alone too)

value = non-null values decoded per second; gbps = algorithmic bytes (encoded page bytes read +
decoded values / offsets / bytes written + level bytes written) / launch time. cpu = the oracle
(value-at-a-time restatement of the reference readers, 1 thread) on a bounded page sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "parquet-mr_amd"), REPO]

from pqgpu import abi  # noqa: E402
from tools.synth import writer  # noqa: E402

sys.path.insert(0, os.path.join(REPO, "tools"))
import workloads as WL  # noqa: E402

HBM_PEAK_GBS = 8000.0


def gen(name, rows):
    """-> workloads.Workload (column chunks + the values written, for verification)."""
    if name in ("c2_zipf2", "c3_mixed", "c5_levels", "c4_lineitem") or name in WL.C3_PARTS:
        return WL.generate(name, rows)
    rng = np.random.default_rng(7)
    E = WL.Expected
    if name == "c1_plain_i32":
        v = np.random.default_rng(1).integers(-2**31, 2**31 - 1, size=rows, dtype=np.int64).astype(np.int32)
        return WL.Workload(name, [writer.write_column_chunk(abi.INT32, v, abi.PLAIN)], [E(v)])
    if name.startswith("str_"):
        enc = {"str_plain": abi.PLAIN, "str_dict": abi.RLE_DICTIONARY, "str_dict_opt": abi.RLE_DICTIONARY,
               "str_dict_16k": abi.RLE_DICTIONARY, "str_dlba": abi.DELTA_LENGTH_BYTE_ARRAY,
               "str_dba": abi.DELTA_BYTE_ARRAY}[name]
        if enc == abi.RLE_DICTIONARY:
            # str_dict: 1,000 entries, required; str_dict_opt: the same with 10 % nulls (V1 pages, parquet-mr's
            # default writer); str_dict_16k: 16,384 entries (past the 2,048-entry / 32 KiB LDS staging)
            card = 16384 if name == "str_dict_16k" else 1000
            dl = WL.nulls(rows, 0.1, 9) if name == "str_dict_opt" else None
            nv = int(dl.sum()) if dl is not None else rows
            words = writer.BinaryValues.random(card, 4, 32, seed=3)
            runs = np.minimum(rng.zipf(1.5, size=nv), 4096)
            ids = np.repeat(rng.integers(0, card, size=runs.size), runs)[:nv]
            ids_fa, order = writer.first_appearance_ids(ids)
            wl = [words[int(o)] for o in order]
            dwords = writer.BinaryValues(np.concatenate([[0], np.cumsum([len(x) for x in wl])]),
                                         np.frombuffer(b"".join(wl), dtype=np.uint8))
            ch = writer.write_dict_column_from_ids(abi.BYTE_ARRAY, dwords, ids_fa, def_levels=dl,
                                                   max_def=1 if dl is not None else 0)
            return WL.Workload(name, [ch], [E(WL.binary_take(wl, ids_fa), dl)])
        if enc == abi.DELTA_BYTE_ARRAY:
            # sorted keys with shared prefixes
            keys = np.sort(rng.integers(0, 10**12, size=rows))
            s = np.char.add(b"https://example.org/item/", np.char.zfill(keys.astype("S12"), 12))
            lens = np.char.str_len(s)
            offs = np.concatenate([[0], np.cumsum(lens)])
            data = np.frombuffer(b"".join(s.tolist()), dtype=np.uint8)
            v = writer.BinaryValues(offs, data)
            return WL.Workload(name, [writer.write_column_chunk(abi.BYTE_ARRAY, v, enc)], [E(v)])
        v = writer.BinaryValues.random(rows, 4, 32, seed=5)
        return WL.Workload(name, [writer.write_column_chunk(abi.BYTE_ARRAY, v, enc)], [E(v)])
    if name == "plain_f64":  # PLAIN doubles, required (k_plain's copy)
        v = rng.standard_normal(rows)
        return WL.Workload(name, [writer.write_column_chunk(abi.DOUBLE, v, abi.PLAIN)], [E(v)])
    if name == "bss_f64":
        v = rng.standard_normal(rows)
        return WL.Workload(name, [writer.write_column_chunk(abi.DOUBLE, v, abi.BYTE_STREAM_SPLIT)], [E(v)])
    if name == "c2_snappy":   # the headline pages, SNAPPY-compressed (parquet-mr's default codec)
        w = WL.c2(rows)
        return WL.Workload(name, [writer.snappy_chunk(w.chunks[0])], w.expect)
    if name == "plain_i64_snappy":  # int64 random walk, PLAIN pages, SNAPPY
        walk = np.cumsum(rng.integers(-100, 1000, size=rows)).astype(np.int64)
        return WL.Workload(name, [writer.snappy_chunk(writer.write_column_chunk(abi.INT64, walk, abi.PLAIN))], [E(walk)])
    if name == "c2_zstd":     # the headline pages, ZSTD-compressed at parquet-mr's default level 3
        w = WL.c2(rows)
        return WL.Workload(name, [writer.zstd_chunk(w.chunks[0])], w.expect)
    if name == "plain_i64_zstd":  # int64 random walk, PLAIN pages, ZSTD level 3
        walk = np.cumsum(rng.integers(-100, 1000, size=rows)).astype(np.int64)
        return WL.Workload(name, [writer.zstd_chunk(writer.write_column_chunk(abi.INT64, walk, abi.PLAIN))], [E(walk)])
    if name == "plain_i64_lz4":  # int64 random walk, PLAIN pages, LZ4_RAW
        walk = np.cumsum(rng.integers(-100, 1000, size=rows)).astype(np.int64)
        return WL.Workload(name, [writer.lz4_raw_chunk(writer.write_column_chunk(abi.INT64, walk, abi.PLAIN))], [E(walk)])
    if name == "c2_lz4":
        w = WL.c2(rows)
        return WL.Workload(name, [writer.lz4_raw_chunk(w.chunks[0])], w.expect)
    if name == "plain_i64_gzip":  # int64 random walk, PLAIN pages, GZIP (zlib level 6, Hadoop's default)
        walk = np.cumsum(rng.integers(-100, 1000, size=rows)).astype(np.int64)
        return WL.Workload(name, [writer.gzip_chunk(writer.write_column_chunk(abi.INT64, walk, abi.PLAIN))], [E(walk)])
    if name == "c2_gzip":
        w = WL.c2(rows)
        return WL.Workload(name, [writer.gzip_chunk(w.chunks[0])], w.expect)
    if name == "delta_i64":
        walk = np.cumsum(rng.integers(-100, 1000, size=rows)).astype(np.int64)
        return WL.Workload(name, [writer.write_column_chunk(abi.INT64, walk, abi.DELTA_BINARY_PACKED)], [E(walk)])
    if name == "delta_i32":  # int32 random walk (the 4-byte DELTA path: 32-bit unpack, sums and scan)
        walk = np.cumsum(rng.integers(-100, 1000, size=rows)).astype(np.int32)
        return WL.Workload(name, [writer.write_column_chunk(abi.INT32, walk, abi.DELTA_BINARY_PACKED)], [E(walk)])
    if name == "delta_i64_2048":  # the same values in DuckDB's DELTA configuration (blocks of 2048, 8 miniblocks)
        walk = np.cumsum(rng.integers(-100, 1000, size=rows)).astype(np.int64)
        return WL.Workload(name, [writer.write_column_chunk(abi.INT64, walk, abi.DELTA_BINARY_PACKED, delta_block=2048,
                                                            delta_miniblocks=8)], [E(walk)])
    raise ValueError(name)


def algo_bytes(batch, cols):
    enc = int(batch.pages["size"].sum()) + sum(int(c["dict_size"]) for c in batch.columns if c["dict_offset"] >= 0)
    out = 0
    for i, cd in enumerate(batch.columns):
        n = cols[i].n_values
        if cd["physical_type"] == abi.BYTE_ARRAY:
            out += 8 * (n + 1) + int(cols[i].offsets()[-1].item())
        else:
            out += n * abi.elem_width(cd["physical_type"], cd["type_length"])
        out += batch.column_slots[i] * ((cd["max_def"] > 0) + (cd["max_rep"] > 0))
    return enc, out


def cpu_sample(chunks, max_pages, budget_s):
    from oracle import pqref
    sub = []
    for ch in chunks:
        c = writer.ColumnChunk(**{k: getattr(ch, k) for k in ("physical_type", "max_rep", "max_def", "type_length",
                                                               "dict_page", "dict_num_values", "dict_encoding")})
        c.pages = ch.pages[:max_pages]
        c.dict_codec, c.dict_uncompressed_size = ch.dict_codec, ch.dict_uncompressed_size
        sub.append(c)
    t_unz, label = 0.0, ""
    if any(p.codec for c in sub for p in c.pages):
        # SNAPPY / ZSTD / LZ4_RAW / GZIP: the oracle decompresses the pages (C restatements of the formats), timed too
        import copy
        fns = {writer.SNAPPY: pqref.snappy_decompress, writer.ZSTD: pqref.zstd_decompress,
               writer.LZ4_RAW: pqref.lz4_raw_decompress, writer.GZIP: pqref.gzip_decompress}
        codec_name = {writer.SNAPPY: "Snappy", writer.ZSTD: "ZSTD", writer.LZ4_RAW: "LZ4_RAW", writer.GZIP: "GZIP"}[next(p.codec for c in sub for p in c.pages if p.codec)]

        def unz(c):
            c = copy.deepcopy(c)
            if c.dict_codec:
                c.dict_page = fns[c.dict_codec](c.dict_page, c.dict_uncompressed_size)
                c.dict_codec = 0
            for p in c.pages:
                if p.codec:
                    lv = p.rl_byte_length + p.dl_byte_length if p.version == 2 else 0
                    p.body = p.body[:lv] + fns[p.codec](p.body[lv:], p.uncompressed_size - lv)
                    p.codec = 0
            return c
        t0, zr = time.perf_counter(), 0
        while True:
            plain = [unz(c) for c in sub]
            zr += 1
            if time.perf_counter() - t0 >= budget_s / 2:
                break
        t_unz = (time.perf_counter() - t0) / zr
        sub, label = plain, f" + {codec_name} decompression {t_unz * 1e3:.1f} ms per rep"
    b = writer.build_batch(sub)
    t0 = time.perf_counter()
    reps = 0
    while True:
        r = pqref.decode_batch(b)
        assert r.code == 0, r.status
        reps += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    nv = sum(c["n_values"] for c in r.columns)
    return {"values_per_s": nv / (dt / reps + t_unz), "cores": 1, "kind": "port",
            "sample": f"first {max_pages} pages of every column, {reps} reps, {dt:.1f} s{label}"}


C5_SCHEMA = [(-1, abi.OPTIONAL), (0, abi.REPEATED), (1, abi.OPTIONAL)]  # optional group list (repeated element: optional int64)


def c5_assemble(dec, cols, batch):
    """Record assembly of the C5 column (RecordReaderImplementation.read's records in columnar form)."""
    return dec.assemble_schema(C5_SCHEMA, [(2, cols[0].def_levels, cols[0].rep_levels, batch.column_slots[0])])


def c5_verify_assembly(got, work, dev):
    import torch
    lens, null_list = work.lists["lens"], work.lists["null_list"]
    assert got["records"] == lens.size
    assert torch.equal(got["nodes"][0]["validity"], torch.from_numpy((~null_list).astype(np.uint8)).to(dev)), "list validity"
    offs = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)).to(dev)
    assert torch.equal(got["nodes"][1]["offsets"], offs), "list offsets"
    dl = work.expect[0].def_levels
    assert torch.equal(got["nodes"][2]["validity"], torch.from_numpy((dl[dl >= 2] == 3).astype(np.uint8)).to(dev)), \
        "element validity"


def run(name, rows, steps, warmup, cpu_budget, check=True):
    import torch
    from pqgpu import decoder as D
    t0 = time.perf_counter()
    work = gen(name, rows)
    chunks = work.chunks
    compressed = any(p.codec for ch in chunks for p in ch.pages)
    t_gen = time.perf_counter() - t0
    dec = D.Decoder(0)
    # A/B runs: PQGPU_DISPATCH="key=value,..." (abi.DISPATCH_* keys, e.g. 5=0: levels first for V2 columns)
    for kv in filter(None, os.environ.get("PQGPU_DISPATCH", "").split(",")):
        k, v = kv.split("=")
        dec.set_dispatch(int(k), int(v))
    if compressed:  # SNAPPY / ZSTD: every timed step decompresses on the GPU, then decodes
        dbatch = dec.upload_chunks(chunks)
        batch = dbatch.batch
    else:
        batch = writer.build_batch(chunks)
        dbatch = dec.upload(batch)
    cols, st = dec.decode(dbatch)  # sizes BYTE_ARRAY buffers, first full decode
    if check:
        WL.verify(cols, work, "decode")
    plan = dec.plan(dbatch, cols)
    plan.launch()
    rc, st = plan.sync()
    assert rc == 0, st.message
    if check:
        WL.verify(cols, work, "first plan launch")
    for _ in range(warmup):
        plan.launch()
    rc, st = plan.sync()
    assert rc == 0, st.message
    assemble = name == "c5_levels"
    if assemble:
        c5_verify_assembly(c5_assemble(dec, cols, batch), work, dec.device)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    torch.cuda.synchronize()
    ev[0].record(dec.stream)
    for k in range(steps):
        dec.decompress(dbatch)
        plan.launch()
        if assemble:  # the step includes the record assembly (synchronous: levels must be decoded)
            got = c5_assemble(dec, cols, batch)
        ev[k + 1].record(dec.stream)
    torch.cuda.synchronize()
    rc, st = plan.sync()
    assert rc == 0, st.message
    if check:
        WL.verify(cols, work, "after the timed launches")
    asm = None
    if assemble:
        c5_verify_assembly(got, work, dec.device)
        ea = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        torch.cuda.synchronize()
        ea[0].record(dec.stream)
        for _ in range(steps):
            got = c5_assemble(dec, cols, batch)
        ea[1].record(dec.stream)
        torch.cuda.synchronize()
        a_ms = ea[0].elapsed_time(ea[1]) / steps
        n_sl = batch.column_slots[0]
        out_b = sum(int(x["validity"].numel()) if x["validity"] is not None else 8 * int(x["offsets"].numel())
                    for x in got["nodes"])
        asm = {"assembly_ms": a_ms, "records": got["records"], "records_per_s": got["records"] / (a_ms / 1e3),
               "assembly_bytes": 2 * n_sl + out_b, "assembly_gbps": (2 * n_sl + out_b) / (a_ms / 1e3) / 1e9,
               "verified": "list validity / offsets and element validity == the generated list structure"}
    ms = float(np.mean([ev[k].elapsed_time(ev[k + 1]) for k in range(steps)]))
    nvals = sum(c.n_values for c in cols)
    nslots = sum(batch.column_slots)
    enc, out = algo_bytes(batch, cols)
    gbps = (enc + out) / (ms / 1e3) / 1e9
    res = {"workload": name, "rows": rows, "columns": len(batch.columns), "pages": batch.n_pages,
           "values": nvals, "slots": nslots, "ms_per_launch": ms, "values_per_s": nvals / (ms / 1e3),
           "encoded_bytes": enc, "output_bytes": out, "gbps": gbps, "hbm_frac": gbps / HBM_PEAK_GBS,
           "kernels_per_launch": plan.kernel_count, "input_gen_s": t_gen,
           "verified": "decoded columns == generated values (decode, first plan launch, after the timed launches)"}
    if asm:
        res["step"] = "plan launch (levels + values) + pqg_assemble_schema"
        res["records_per_s"] = asm["records"] / (ms / 1e3)
        res["assembly"] = asm
        res["gbps"] = (enc + out + asm["assembly_bytes"]) / (ms / 1e3) / 1e9
        res["hbm_frac"] = res["gbps"] / HBM_PEAK_GBS
    if compressed:
        comp = sum(len(p.body) for ch in chunks for p in ch.pages) + sum(len(ch.dict_page or b"") for ch in chunks)
        ev2 = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        torch.cuda.synchronize()
        ev2[0].record(dec.stream)
        for _ in range(steps):
            dec.decompress(dbatch)
        ev2[1].record(dec.stream)
        torch.cuda.synchronize()
        sms = ev2[0].elapsed_time(ev2[1]) / steps
        codec = {writer.SNAPPY: "snappy", writer.ZSTD: "zstd", writer.LZ4_RAW: "lz4_raw", writer.GZIP: "gzip"}[next(p.codec for ch in chunks for p in ch.pages if p.codec)]
        res.update({"compressed_bytes": comp, f"{codec}_ms": sms,
                    f"{codec}_gbps_uncompressed": enc / (sms / 1e3) / 1e9})
    if name == "c1_plain_i32":
        t1 = time.perf_counter()
        rc2, st2, res2, _ = dec.decode_host(batch)
        e2e = time.perf_counter() - t1
        assert rc2 == 0
        res["e2e_host_values_per_s"] = nvals / e2e
    if cpu_budget > 0:
        res["cpu"] = cpu_sample(chunks, 50, cpu_budget)
    plan.close()
    dec.close()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("workloads", nargs="*", default=["c1_plain_i32", "c2_zipf2", "c3_mixed", "c5_levels", "str_plain",
                                                     "str_dict", "str_dict_opt", "str_dict_16k", "str_dlba", "str_dba",
                                                     "plain_f64", "bss_f64", "delta_i64", "delta_i32",
                                                     "delta_i64_2048"])
    ap.add_argument("--rows", type=int, default=None, help="override the per-workload row count")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-budget", type=float, default=2.0)
    ap.add_argument("--gen-only", action="store_true")
    ap.add_argument("--no-verify", action="store_true", help="diagnostic builds that skip work: no output checks")
    args = ap.parse_args()
    default_rows = {"c1_plain_i32": 1_000_000, "c2_zipf2": 100_000_000, "c3_mixed": 100_000_000,
                    "c5_levels": 100_000_000, "str_plain": 20_000_000, "str_dict": 20_000_000,
                    "str_dlba": 20_000_000, "str_dba": 20_000_000, "bss_f64": 100_000_000, "plain_f64": 100_000_000, "delta_i64": 100_000_000, "delta_i32": 100_000_000,
                    "delta_i64_2048": 100_000_000,
                    "c2_snappy": 100_000_000, "plain_i64_snappy": 100_000_000,
                    "c2_zstd": 100_000_000, "plain_i64_zstd": 100_000_000,
                    "c2_lz4": 100_000_000, "plain_i64_lz4": 100_000_000,
                    "c2_gzip": 100_000_000, "plain_i64_gzip": 100_000_000,
                    "c4_lineitem": 8_000_000, "c3_delta": 100_000_000, "c3_double": 100_000_000,
                    "str_dict_opt": 20_000_000, "str_dict_16k": 20_000_000,
                    "c3_strings": 100_000_000}
    for w in args.workloads:
        rows = args.rows or default_rows[w]
        if args.gen_only:
            t0 = time.perf_counter()
            b = writer.build_batch(gen(w, rows).chunks)
            print(json.dumps({"workload": w, "rows": rows, "pages": b.n_pages, "bytes": int(b.data.size),
                              "gen_s": time.perf_counter() - t0}), flush=True)
            continue
        print(json.dumps(run(w, rows, args.steps, args.warmup, args.cpu_budget, not args.no_verify)), flush=True)


if __name__ == "__main__":
    main()
