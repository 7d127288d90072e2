"""Diagnostic: where the ZSTD kernel's cycles go (diagnostic build, -DPQG_DIAG): per job, s_memtime
cycles in literal (Huffman) decoding, sequence tables, the sequence loop, batch execution inside it,
long sequences, the whole job; sequence and literal counts. Runs the suite's plain_i64_zstd input.
Usage: PQGPU_LIB=abx/libdiag.so python tools/diag_zstd.py [rows]"""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "parquet-mr_amd"), os.path.join(REPO, "tools"), REPO]
import torch  # noqa: E402

import bench_suite  # noqa: E402
from pqgpu import decoder as D, native  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
work = bench_suite.gen("plain_i64_zstd", rows)
dec = D.Decoder(0)
db = dec.upload_chunks(work.chunks)
n_jobs = sum(1 for ch in work.chunks for p in ch.pages if p.codec)
buf = torch.zeros(max(n_jobs, 1) * 12 + 64, dtype=torch.int64, device="cuda")
L = native.lib()
L.pqg_diag_zstd_set.argtypes = [C.c_void_p]
assert L.pqg_diag_zstd_set(buf.data_ptr()) == 0
zq = torch.zeros(max(n_jobs, 1) * 6 + 64, dtype=torch.int64, device="cuda")
if hasattr(L, "pqg_diag_zq_set"):
    L.pqg_diag_zq_set.argtypes = [C.c_void_p]
    assert L.pqg_diag_zq_set(zq.data_ptr()) == 0
dec.decompress(db)
torch.cuda.synchronize()
q = zq[: n_jobs * 6].view(n_jobs, 6).cpu().numpy().astype(np.float64)
if q[:, 0].sum():
    print(f"pre-pass (k_zstd_seq, one lane per job): mean job cycles {q[:, 0].mean():.0f}, tables {q[:, 1].mean():.0f}, "
          f"sequence loops {q[:, 2].mean():.0f}; sequences {q[:, 3].mean():.0f}, re-centrings {q[:, 4].mean():.1f}, "
          f"blocks {q[:, 5].mean():.1f}; loop cycles per sequence {q[:, 2].sum() / max(q[:, 3].sum(), 1):.0f}")
a = buf[: n_jobs * 12].view(n_jobs, 12).cpu().numpy().astype(np.float64)
names = ["literals", "seq tables", "seq loop", "  batches", "  long seqs", "job", "sequences", "literal bytes",
         "  state reads", "  extra bits", "  state updates", "  rest"]
tot = a[:, 5].sum()
print(f"jobs {n_jobs}, mean job cycles {a[:, 5].mean():.0f}")
for i, nm in enumerate(names):
    print(f"{nm:14s} sum {a[:, i].sum():16.0f}  per job {a[:, i].mean():12.0f}" +
          (f"  {100 * a[:, i].sum() / tot:5.1f} %" if i < 6 or i >= 8 else ""))
print(f"cycles per sequence (loop): {a[:, 2].sum() / max(a[:, 6].sum(), 1):.0f}, "
      f"per batch-executed sequence: {a[:, 3].sum() / max(a[:, 6].sum(), 1):.0f}, "
      f"literal cycles per byte: {a[:, 0].sum() / max(a[:, 7].sum(), 1):.1f}")
