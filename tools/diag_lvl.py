"""Diagnostic: where k_levels' cycles go (diagnostic build, -DPQG_DIAG): per page, s_memtime cycles of the
def-level decode's phases summed over its windows — window pre-decode + table stores, binary lifting,
chain batches (run table), tile expansion — and the window count.
Usage: PQGPU_LIB=abx/libdiag.so python tools/diag_lvl.py [null_frac] [rows]"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "parquet-mr_amd"), REPO]
import torch  # noqa: E402

from pqgpu import abi, decoder as D, native  # noqa: E402
from tools.synth import writer  # noqa: E402

frac = float(sys.argv[1]) if len(sys.argv) > 1 else 0.1
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
dl = (np.random.default_rng(8).random(rows) >= frac).astype(np.uint8)
n = int(dl.sum())
ch = writer.write_column_chunk(abi.DOUBLE, np.zeros(n), abi.PLAIN, def_levels=dl, max_def=1, version=2)
batch = writer.build_batch([ch])
dec = D.Decoder(0)
db = dec.upload(batch)
cols, st = dec.decode(db)
plan = dec.plan(db, cols)
n_pages = batch.n_pages
wph = torch.zeros(n_pages * 8, dtype=torch.int64, device="cuda")
L = native.lib()
L.pqg_diag_wph_set.argtypes = [C.c_void_p]
for _ in range(3):
    plan.launch()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(dec.stream)
for _ in range(5):
    plan.launch()
e1.record(dec.stream)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
assert L.pqg_diag_wph_set(C.c_void_p(wph.data_ptr())) == 0
plan.launch()
torch.cuda.synchronize()
assert L.pqg_diag_wph_set(None) == 0
ph = wph.view(-1, 8).cpu().numpy()[:, :5].astype(np.float64)
tot = ph[:, :4].sum(axis=0)
win = ph[:, 4].sum()
names = ["predecode", "lifting", "chain", "expand"]
print(json.dumps({"null_frac": frac, "rows": rows, "pages": n_pages, "plan_ms": ms, "windows": win,
                  "cycles_per_window": {k: tot[i] / win for i, k in enumerate(names)},
                  "share": {k: tot[i] / tot.sum() for i, k in enumerate(names)},
                  "cycles_per_page_mean": float(ph[:, :4].sum(axis=1).mean())}), flush=True)
plan.close()
