"""Diagnostic: per-kernel time of the C2 plan with output stores disabled (libpqgpu_diag.so).
Usage: PQGPU_LIB=.../libpqgpu_diag.so rocprofv3 --kernel-trace --stats -- python tools/nostore_bench.py [nostore]"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "parquet-mr_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

import bench  # noqa: E402
from pqgpu import decoder as D, native  # noqa: E402
from tools.synth import writer  # noqa: E402

nostore = len(sys.argv) > 1 and sys.argv[1] == "nostore"
chunk, dv, ids = bench.make_c2(100_000_000)
batch = writer.build_batch([chunk])
dec = D.Decoder(0)
plan = dec.plan(dec.upload(batch))
L = native.lib()
L.pqg_diag_nostore_set.argtypes = [C.c_int]
assert L.pqg_diag_nostore_set(1 if nostore else 0) == 0
for _ in range(10):
    plan.launch()
torch.cuda.synchronize()
print("done", nostore)
