"""Diagnostic: level-decode time vs null pattern (run structure) and page version."""
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
rows = 20_000_000
for frac, ver in [(0.0, 2), (0.1, 2), (0.1, 1), (0.5, 2), (0.01, 2)]:
    dl = (np.random.default_rng(8).random(rows) >= frac).astype(np.uint8)
    n = int(dl.sum())
    ch = writer.write_column_chunk(abi.DOUBLE, np.zeros(n), abi.PLAIN, def_levels=dl, max_def=1, version=ver)
    batch = writer.build_batch([ch])
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
    lvl_bytes = sum(len(p.body) - 8 * (p.num_values - p.num_nulls) for p in ch.pages)
    print(json.dumps({"null_frac": frac, "version": ver, "pages": batch.n_pages, "ms": ms, "level_bytes": lvl_bytes}),
          flush=True)
    plan.close()
