"""Diagnostic: per-tile timeline of k_bin_plain (diagnostic build, -DPQG_DIAG): s_memrealtime at the
tile's start, after its walk, after its look-back, at its end; look-back polls; whether the guess held.
Usage: PQGPU_LIB=abx/libdiag.so python tools/diag_binplain.py [workload] [rows]"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "parquet-mr_amd"), os.path.join(REPO, "tools"), REPO]
import torch  # noqa: E402

import bench_suite  # noqa: E402
from pqgpu import decoder as D, native  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "str_plain"
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000_000
work = bench_suite.gen(name, rows)
dec = D.Decoder(0)
db = dec.upload(work.batch) if hasattr(work, "batch") else dec.upload_chunks(work.chunks)
plan = dec.plan(db)
plan.launch()
plan.sync()
n_tiles = int(sum((int(p["size"]) + 2047) // 2048 for p in db.batch.pages)) + 64
buf = torch.zeros(n_tiles * 8, dtype=torch.int64, device="cuda")
L = native.lib()
L.pqg_diag_bp_set.argtypes = [C.c_void_p]
assert L.pqg_diag_bp_set(buf.data_ptr()) == 0
plan.launch()
torch.cuda.synchronize()
assert L.pqg_diag_bp_set(None) == 0
a = buf.view(-1, 8).cpu().numpy()
a = a[a[:, 0] != 0].astype(np.float64)
t0 = a[:, 0].min()
st, wk, lb, en = (a[:, 0] - t0) / 100, (a[:, 1] - t0) / 100, (a[:, 2] - t0) / 100, (a[:, 3] - t0) / 100
pct = [0, 10, 50, 90, 99, 100]
print("tiles", len(a), "span_us", round(en.max(), 1))
print("start_us", np.percentile(st, pct).round(1).tolist())
print("walk_us", np.percentile(wk - st, pct).round(1).tolist())
print("lookback_us", np.percentile(lb - wk, pct).round(1).tolist())
print("emit_us", np.percentile(en - lb, pct).round(1).tolist())
gs = (a[:, 4] - t0) / 100
print("guess_us", np.percentile(gs - st, pct).round(1).tolist(), "walk_after_guess_us", np.percentile(wk - gs, pct).round(1).tolist())
print("guess_held", a[:, 5].mean())
edges = np.arange(0, en.max() + 50, 50.0)
print("alive per 50us", [int(((st < b + 50) & (en > b)).sum()) for b in edges][:40])
