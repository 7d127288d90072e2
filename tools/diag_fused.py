"""Diagnostic: timeline of one k_dict_fused launch (diagnostic build, -DPQG_DIAG).
Walkers stamp s_memrealtime (100 MHz, chip-wide) at walk start and at publish; expansion chunks at
start, when their page's flag is seen, and at the end. Prints the distributions and how many chunks
spin / store over time.
Usage: PQGPU_LIB=abx/libdiag.so python tools/diag_fused.py [zipf] [out.json]"""
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
out = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out/diag_fused.json"
chunk, dv, ids = bench.make_c2(100_000_000, a=zipf)
batch = writer.build_batch([chunk])
dec = D.Decoder(0)
plan = dec.plan(dec.upload(batch))
n_pages = batch.n_pages
max_chunks = n_pages * 16
wrt = torch.zeros(n_pages * 4, dtype=torch.int64, device="cuda")
xrt = torch.zeros(max_chunks * 4, dtype=torch.int64, device="cuda")
wph = torch.zeros(n_pages * 8, dtype=torch.int64, device="cuda")
L = native.lib()
L.pqg_diag_rt_set.argtypes = [C.c_void_p, C.c_void_p]
L.pqg_diag_wph_set.argtypes = [C.c_void_p]
for _ in range(3):
    plan.launch()
torch.cuda.synchronize()
res = {"zipf": zipf, "runs": []}
for rep in range(3):
    wrt.zero_()
    xrt.zero_()
    torch.cuda.synchronize()
    assert L.pqg_diag_rt_set(wrt.data_ptr(), xrt.data_ptr()) == 0
    assert L.pqg_diag_wph_set(C.c_void_p(wph.data_ptr())) == 0
    plan.launch()
    torch.cuda.synchronize()
    assert L.pqg_diag_rt_set(None, None) == 0
    assert L.pqg_diag_wph_set(None) == 0
    ph = wph.view(-1, 8).cpu().numpy().astype(np.float64)
    w = wrt.view(-1, 4).cpu().numpy().astype(np.float64)
    x = xrt.view(-1, 4).cpu().numpy()
    x = x[x[:, 0] != 0]
    xt = x[:, :3].astype(np.float64)
    t0 = min(w[:, 0].min(), xt[:, 0].min())
    w = (w - t0) / 100.0   # us
    xt = (xt - t0) / 100.0
    end = max(w[:, 1].max(), xt[:, 2].max())
    pct = [0, 10, 50, 90, 100]
    spin = xt[:, 1] - xt[:, 0]
    body = xt[:, 2] - xt[:, 1]
    # chunks storing / spinning per 5 us bucket
    edges = np.arange(0, end + 5, 5.0)
    storing = [int(((xt[:, 1] < b + 5) & (xt[:, 2] > b)).sum()) for b in edges]
    spinning = [int(((xt[:, 0] < b + 5) & (xt[:, 1] > b)).sum()) for b in edges]
    walking = [int(((w[:, 0] < b + 5) & (w[:, 1] > b)).sum()) for b in edges]
    r = {"kernel_us": end, "chunks": int(len(xt)),
         "walk_start_us": np.percentile(w[:, 0], pct).tolist(), "walk_pub_us": np.percentile(w[:, 1], pct).tolist(),
         "walk_dur_us": np.percentile(w[:, 1] - w[:, 0], pct).tolist(),
         "walk_stage_us": np.percentile(w[:, 2] - w[:, 0], pct).tolist(),
         "walk_chain_us": np.percentile(w[:, 3] - w[:, 2], pct).tolist(),
         "walk_release_us": np.percentile(w[:, 1] - w[:, 3], pct).tolist(),
         "chunk_start_us": np.percentile(xt[:, 0], pct).tolist(), "chunk_spin_us": np.percentile(spin, pct).tolist(),
         "chunk_body_us": np.percentile(body, pct).tolist(), "chunk_end_us": np.percentile(xt[:, 2], pct).tolist(),
         "list_walk_kcyc_pre_chain_emit_mean": (ph[:, :3].mean(0) / 1e3).tolist(),
         "list_walk_windows_batches_runs_mean": ph[:, 3:6].mean(0).tolist(),
         "bucket_us": 5.0, "walking": walking, "spinning": spinning, "storing": storing}
    res["runs"].append(r)
    print(json.dumps({k: (np.round(v, 1).tolist() if isinstance(v, list) else v) for k, v in r.items()}), flush=True)
os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
json.dump(res, open(out, "w"), indent=1)
