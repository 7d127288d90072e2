"""Diagnostic: k_dict<8> launch time vs number of C2 pages in the launch.

Separates per-wave latency (time flat in the page count while waves < slots) from
shared-resource contention (time growing with concurrent waves). With the diag
library (PQGPU_LIB=.../libpqgpu_diag.so) it also reports per-wave durations.
Usage: python tools/scale_pages.py [zipf] [out.json] [nostore]
"""
import copy
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "parquet-mr_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from pqgpu import decoder as D, native  # noqa: E402
from tools.synth import writer  # noqa: E402

zipf = float(sys.argv[1]) if len(sys.argv) > 1 else 1.5
out = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/scale_pages.json"
nostore = len(sys.argv) > 3 and sys.argv[3] == "nostore"
diag = os.environ.get("PQGPU_LIB", "").endswith("_diag.so")
chunk, dv, ids = bench.make_c2(100_000_000, a=zipf)
dec = D.Decoder(0)
L = native.lib()
res = {"zipf": zipf, "nostore": nostore, "diag": diag, "rows": []}
for k in (1, 4, 64, 256, 1024, 2048, 3072, 4096, 5000):
    sub = copy.copy(chunk)
    sub.pages = chunk.pages[:k]
    batch = writer.build_batch([sub])
    plan = dec.plan(dec.upload(batch))
    buf = None
    if diag:
        buf = torch.zeros(batch.n_pages * 8, dtype=torch.int64, device="cuda")
        L.pqg_diag_set.argtypes = [C.c_void_p]
        assert L.pqg_diag_set(buf.data_ptr()) == 0
        L.pqg_diag_nostore_set.argtypes = [C.c_int]
        assert L.pqg_diag_nostore_set(1 if nostore else 0) == 0
    for _ in range(3):
        plan.launch()
    rc, st = plan.sync()
    assert rc == 0, st.message
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(11)]
    ev[0].record(dec.stream)
    for i in range(10):
        plan.launch()
        ev[i + 1].record(dec.stream)
    torch.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(10)]
    row = {"pages": k, "launch_ms_min": min(ms), "launch_ms_med": float(np.median(ms))}
    if diag:
        d = buf.view(-1, 8).cpu().numpy().astype(np.float64)
        row["dur_us_pct"] = np.percentile((d[:, 1] - d[:, 0]) / 100.0, [0, 50, 90, 100]).tolist()
        row["walk_kcyc_med"] = float(np.median(d[:, 2]) / 1e3)
        row["exp_kcyc_med"] = float(np.median(d[:, 4]) / 1e3)
        L.pqg_diag_set(None)
    print(json.dumps(row), flush=True)
    res["rows"].append(row)
    plan.close()
os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
json.dump(res, open(out, "w"), indent=1)
