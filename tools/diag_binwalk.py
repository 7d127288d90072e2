"""Diagnostic: PLAIN BYTE_ARRAY decode time vs string length and page count (per-kernel times
come from rocprofv3 around this script)."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "parquet-mr_amd"), REPO]
import torch  # noqa: E402
from pqgpu import abi, decoder as D  # noqa: E402
from tools.synth import writer  # noqa: E402

dec = D.Decoder(0)
for (lo, hi, rows, page_rows) in [(0, 0, 4_000_000, 20000), (4, 32, 4_000_000, 20000), (100, 200, 1_000_000, 5000),
                                  (4, 32, 4_000_000, 2000)]:
    v = writer.BinaryValues.random(rows, lo, hi, seed=1)
    batch = writer.build_batch([writer.write_column_chunk(abi.BYTE_ARRAY, v, abi.PLAIN, page_rows=page_rows)])
    db = dec.upload(batch)
    cols, st = dec.decode(db)
    plan = dec.plan(db, cols)
    plan.launch()
    plan.sync()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(dec.stream)
    for _ in range(5):
        plan.launch()
    e1.record(dec.stream)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    print(json.dumps({"len": [lo, hi], "rows": rows, "pages": batch.n_pages, "ms": ms,
                      "bytes": int(batch.pages["size"].sum()), "gbps": int(batch.pages["size"].sum()) / ms / 1e6}),
          flush=True)
    plan.close()
