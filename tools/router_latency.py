"""Per-call latency of the ParquetReadRouter boundary.

ParquetReadRouter.read (parquet-plugins/.../ParquetReadRouter.java:57-66) is called once per
bit-packed run of at most 504 values. Measures, on the GPU box, through the C ABI with host buffers:
  one run per call       pqg_router_read       (H2D, kernel, D2H, synchronize per run)
  a page's runs per call pqg_router_read_runs  (the same, once per page)
and prints one JSON line per case: calls, mean / p50 / p99 microseconds per call, values per second.
Every result is checked against the oracle's router (pqr_router_read) once before timing.
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "parquet-mr_amd"), REPO]

from pqgpu import decoder as D  # noqa: E402


def page_of_runs(w, n_runs, seed=1):
    """A page section of n_runs bit-packed runs of 504 values (63 groups) at width w, 1-byte gaps
    (the run headers)."""
    rng = np.random.default_rng(seed)
    counts = np.full(n_runs, 504, dtype=np.uint32)
    offs, pos = [], 0
    for c in counts:
        pos += 1
        offs.append(pos)
        pos += int(c) * w // 8
    data = rng.integers(0, 256, size=pos + 8, dtype=np.uint8)
    return data, np.array(offs, dtype=np.uint64), counts


def timed(fn, reps):
    t = []
    for _ in range(reps):
        t0 = time.perf_counter_ns()
        fn()
        t.append((time.perf_counter_ns() - t0) / 1e3)
    t = np.array(t)
    return float(t.mean()), float(np.percentile(t, 50)), float(np.percentile(t, 99))


def main():
    from oracle import pqref
    dec = D.Decoder(0)
    w = 10
    data, offs, counts = page_of_runs(w, 40)   # a 20,160-value page (C2's page size, all packed)
    want = np.concatenate([pqref.router_read(w, data[int(o):].tobytes(), int(c))[0] for o, c in zip(offs, counts)])
    got = dec.router_read_runs(w, data, offs, counts)
    assert np.array_equal(got, want), "pqg_router_read_runs differs from the oracle"
    one = data[int(offs[0]):int(offs[0]) + 504 * w // 8]
    assert np.array_equal(dec.router_read(w, one, 504), want[:504]), "pqg_router_read differs from the oracle"
    for _ in range(50):  # warm up
        dec.router_read(w, one, 504)
        dec.router_read_runs(w, data, offs, counts)
    m, p50, p99 = timed(lambda: dec.router_read(w, one, 504), 2000)
    print(json.dumps({"case": "pqg_router_read, one 504-value run per call", "bit_width": w, "calls": 2000,
                      "us_mean": round(m, 2), "us_p50": round(p50, 2), "us_p99": round(p99, 2),
                      "values_per_s": round(504 / (m * 1e-6)), "us_per_page_of_40_runs": round(40 * m, 1)}),
          flush=True)
    m, p50, p99 = timed(lambda: dec.router_read_runs(w, data, offs, counts), 500)
    print(json.dumps({"case": "pqg_router_read_runs, 40 runs (one page) per call", "bit_width": w, "calls": 500,
                      "us_mean": round(m, 2), "us_p50": round(p50, 2), "us_p99": round(p99, 2),
                      "values_per_s": round(int(counts.sum()) / (m * 1e-6))}), flush=True)


if __name__ == "__main__":
    main()
