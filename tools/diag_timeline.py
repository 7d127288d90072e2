"""Diagnostic: per-wave timeline of k_dict<8> on the C2 workload (libpqgpu_diag.so only)."""
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PQGPU_LIB"] = os.path.join(REPO, "parquet-mr_amd", "pqgpu", "libpqgpu_diag.so")
sys.path.insert(0, os.path.join(REPO, "parquet-mr_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from pqgpu import decoder as D, native  # noqa: E402
from tools.synth import writer  # noqa: E402

zipf = float(sys.argv[1]) if len(sys.argv) > 1 else 1.5
out = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/diag.json"
nostore = len(sys.argv) > 3 and sys.argv[3] == "nostore"
chunk, dv, ids = bench.make_c2(100_000_000, a=zipf)
batch = writer.build_batch([chunk])
dec = D.Decoder(0)
plan = dec.plan(dec.upload(batch))
buf = torch.zeros(batch.n_pages * 8, dtype=torch.int64, device="cuda")
L = native.lib()
L.pqg_diag_set.argtypes = [C.c_void_p]
assert L.pqg_diag_set(buf.data_ptr()) == 0
L.pqg_diag_nostore_set.argtypes = [C.c_int]
assert L.pqg_diag_nostore_set(1 if nostore else 0) == 0
for _ in range(3):
    plan.launch()
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record(dec.stream)
plan.launch()
ev1.record(dec.stream)
torch.cuda.synchronize()
d = buf.view(-1, 8).cpu().numpy().astype(np.float64)
start, end = d[:, 0], d[:, 1]
t0 = start.min()
res = {
    "zipf": zipf, "nostore": nostore, "kernel_ms_event": ev0.elapsed_time(ev1),
    "span_us": (end.max() - t0) / 100.0,  # s_memrealtime: 100 MHz
    "start_us_pct": np.percentile((start - t0) / 100.0, [0, 10, 50, 90, 99, 100]).tolist(),
    "dur_us_pct": np.percentile((end - start) / 100.0, [0, 10, 50, 90, 99, 100]).tolist(),
    "walk_kcyc_pct": np.percentile(d[:, 2] / 1e3, [0, 50, 90, 100]).tolist(),
    "stage_kcyc_pct": np.percentile(d[:, 3] / 1e3, [0, 50, 90, 100]).tolist(),
    "exp_kcyc_pct": np.percentile(d[:, 4] / 1e3, [0, 50, 90, 100]).tolist(),
    "batches_pct": np.percentile(d[:, 5], [0, 50, 100]).tolist(),
    "xcc_counts": np.bincount((d[:, 6].astype(np.int64) >> 32), minlength=8).tolist(),
}
# concurrency profile: waves alive at 20 time points
ts = np.linspace(t0, end.max(), 21)
res["alive"] = [int(((start <= t) & (end > t)).sum()) for t in ts]
print(json.dumps(res, indent=1))
os.makedirs(os.path.dirname(out), exist_ok=True)
json.dump(res, open(out, "w"), indent=1)
