"""Diagnostic: per-page phase cycles of the pointer-jumping walk (libpqgpu_diag.so).
Usage: PQGPU_LIB=.../libpqgpu_diag.so python tools/diag_walk.py [zipf] [out.json]"""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PQGPU_LIB", os.path.join(REPO, "parquet-mr_amd", "pqgpu", "libpqgpu_diag.so"))
sys.path.insert(0, os.path.join(REPO, "parquet-mr_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from pqgpu import decoder as D, native  # noqa: E402
from tools.synth import writer  # noqa: E402

zipf = float(sys.argv[1]) if len(sys.argv) > 1 else 1.5
out = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/diag_walk.json"
chunk, dv, ids = bench.make_c2(100_000_000, a=zipf)
batch = writer.build_batch([chunk])
dec = D.Decoder(0)
plan = dec.plan(dec.upload(batch))
buf = torch.zeros(batch.n_pages * 8, dtype=torch.int64, device="cuda")
L = native.lib()
L.pqg_diag_set.argtypes = [C.c_void_p]
assert L.pqg_diag_set(buf.data_ptr()) == 0
for _ in range(3):
    plan.launch()
torch.cuda.synchronize()
d = buf.view(-1, 8).cpu().numpy().astype(np.float64)
dur = d[:, 1] - d[:, 0]
pct = [0, 10, 50, 90, 99, 100]
res = {"zipf": zipf, "dur_kcyc": np.percentile(dur / 1e3, pct).tolist(),
       "pre_kcyc": np.percentile(d[:, 2] / 1e3, pct).tolist(), "dbl_kcyc": np.percentile(d[:, 3] / 1e3, pct).tolist(),
       "emit_kcyc": np.percentile(d[:, 4] / 1e3, pct).tolist(), "windows": np.percentile(d[:, 5], pct).tolist(),
       "runs": np.percentile(d[:, 6], pct).tolist()}
top = np.argsort(dur)[-5:]
res["slowest"] = [{"page": int(p), "kcyc": dur[p] / 1e3, "pre": d[p, 2] / 1e3, "dbl": d[p, 3] / 1e3,
                   "emit": d[p, 4] / 1e3, "windows": int(d[p, 5]), "runs": int(d[p, 6])} for p in top]
print(json.dumps(res, indent=1))
os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
json.dump(res, open(out, "w"), indent=1)
