"""Recovery from the fused dictionary kernel's wait timeout (pqgpu_kernels.hip SPIN_TIMEOUT_TICKS).

The fused kernel's expansion workgroups wait for the walker workgroups of their pages; HIP does not
promise that walkers are dispatched first. When a wait exceeds the timeout the launch reports
PQG_ERR_TIMEOUT internally and pqg_sync re-runs the plan in split mode (walk, then expansion as a
second launch), which has no inter-workgroup waits; the caller must see the normal, bit-exact result.

The fault is injected, once per launch and deterministically, by a test build of the library
(tests/build/libpqgpu_faultinject.so, built by __graft_entry__.build with -DPQG_FAULT_INJECT): walker
workgroup 0 starts 0.5 s late and the spin timeout is 0.1 s. The check runs in a child process that
loads that build (PQGPU_LIB); the product library is never built with the knob."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INJECT_LIB = os.path.join(REPO, "tests", "build", "libpqgpu_faultinject.so")

CHILD = r"""
import json, sys
import numpy as np, torch
sys.path[:0] = [sys.argv[1] + "/parquet-mr_amd", sys.argv[1] + "/tools", sys.argv[1]]
import workloads as WL
from pqgpu import decoder as D, native
from tools.synth import writer
assert native.LIB_PATH.endswith("libpqgpu_faultinject.so"), native.LIB_PATH
out = {}
chunk, dict_vals, ids = WL.make_c2(2_000_000, 42, 43, 1.5, 1000, 4096, 20000)
exp = torch.from_numpy(dict_vals[ids])
batch = writer.build_batch([chunk])
dec = D.Decoder(0, poison=0xA5)
dbatch = dec.upload(batch)
cols = dec.alloc_columns(batch)
plan = dec.plan(dbatch, cols)
k0 = plan.kernel_count
plan.launch()
rc, st = plan.sync()
out["first"] = {"rc": rc, "fallbacks": plan.timeout_fallbacks, "kernels": plan.kernel_count, "kernels_before": k0,
                "equal": bool(torch.equal(cols[0].typed().cpu(), exp))}
cols[0].values.fill_(0xA5)
plan.launch()
rc, st = plan.sync()
out["second"] = {"rc": rc, "fallbacks": plan.timeout_fallbacks, "equal": bool(torch.equal(cols[0].typed().cpu(), exp))}
plan.close()
# the one-call path (pqg_decode + pqg_sync) recovers the same way
cols2, st2 = dec.decode(dbatch)
out["decode"] = {"equal": bool(torch.equal(cols2[0].typed().cpu(), exp))}
dec.close()
print("RESULT " + json.dumps(out))
"""


@pytest.mark.gpu
def test_timed_out_fused_launch_is_rerun_split_and_bit_exact(tmp_path):
    assert os.path.exists(INJECT_LIB), "build() makes the fault-injection library"
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    env = dict(os.environ, PQGPU_LIB=INJECT_LIB)
    r = subprocess.run([sys.executable, str(script), REPO], env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1]
    res = json.loads(line[7:])
    f = res["first"]
    assert f["rc"] == 0 and f["equal"], res
    assert f["fallbacks"] == 1, res                      # the injected delay did time the launch out
    assert f["kernels"] == f["kernels_before"] + 1, res  # walk + expansion: two launches now
    s = res["second"]
    assert s["rc"] == 0 and s["equal"] and s["fallbacks"] == 1, res  # split mode stays: no further timeout
    assert res["decode"]["equal"], res


CHILD_SEG = r"""
import json, sys
import numpy as np, torch
sys.path[:0] = [sys.argv[1] + "/parquet-mr_amd", sys.argv[1] + "/tools", sys.argv[1]]
from pqgpu import abi, decoder as D, native
from tools.synth import writer
assert native.LIB_PATH.endswith("libpqgpu_faultinject.so"), native.LIB_PATH
vals = writer.BinaryValues.random(60_000, 4, 32, seed=5)
chunk = writer.write_column_chunk(abi.BYTE_ARRAY, vals, abi.PLAIN)  # 3 pages of ~440 KB: segmented
batch = writer.build_batch([chunk])
exp_off = torch.from_numpy(vals.offsets)
exp_data = torch.from_numpy(vals.data[: int(vals.offsets[-1])].copy())
dec = D.Decoder(0, poison=0xA5)
dec.set_dispatch(abi.DISPATCH_PLAIN_ONE_PASS, 0)  # the per-value path: k_bin_walk_seg for few large pages
dbatch = dec.upload(batch)
cols = dec.alloc_columns(batch)
plan = dec.plan(dbatch, cols)
k0 = plan.kernel_count
def same(c):
    off = c.offsets().cpu()
    return bool(torch.equal(off, exp_off)) and bool(torch.equal(c.binary_data[: int(off[-1])].cpu(), exp_data))
out = {}
plan.launch()
rc, st = plan.sync()
out["first"] = {"rc": rc, "fallbacks": plan.timeout_fallbacks, "kernels": plan.kernel_count, "kernels_before": k0,
                "equal": same(cols[0])}
cols[0].binary_data.fill_(0xA5)
plan.launch()
rc, st = plan.sync()
out["second"] = {"rc": rc, "fallbacks": plan.timeout_fallbacks, "equal": same(cols[0])}
plan.close()
dec.close()
print("RESULT " + json.dumps(out))
"""


@pytest.mark.gpu
def test_timed_out_segment_walk_is_rerun_per_page_and_bit_exact(tmp_path):
    """The segmented PLAIN BYTE_ARRAY walk (k_bin_walk_seg): a segment whose predecessor publishes past
    the wait bound reports PQG_ERR_TIMEOUT; pqg_sync re-runs the plan with those pages one wave each
    (k_bin_walk) and the caller sees the normal, bit-exact result. Injected as above: the wave holding
    the first ticket publishes 0.5 s late, the bound is 0.1 s."""
    assert os.path.exists(INJECT_LIB), "build() makes the fault-injection library"
    script = tmp_path / "child_seg.py"
    script.write_text(CHILD_SEG)
    env = dict(os.environ, PQGPU_LIB=INJECT_LIB)
    r = subprocess.run([sys.executable, str(script), REPO], env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1]
    res = json.loads(line[7:])
    f = res["first"]
    assert f["rc"] == 0 and f["equal"], res
    assert f["fallbacks"] == 1, res                  # the injected delay did time the segment walk out
    assert f["kernels"] == f["kernels_before"], res  # k_bin_walk_seg replaced by one k_bin_walk launch
    s = res["second"]
    assert s["rc"] == 0 and s["equal"] and s["fallbacks"] == 1, res  # per-page mode stays: no further timeout


CHILD_DD = r"""
import json, sys
import numpy as np, torch
sys.path[:0] = [sys.argv[1] + "/parquet-mr_amd", sys.argv[1] + "/tools", sys.argv[1]]
from pqgpu import abi, decoder as D, native
from tools.synth import writer
assert native.LIB_PATH.endswith("libpqgpu_faultinject.so"), native.LIB_PATH
words = [b"DELIVER IN PERSON", b"COLLECT COD", b"NONE", b"TAKE BACK RETURN", b"R", b"", b"AIR", b"MAIL"]
ids = np.random.default_rng(3).integers(0, len(words), size=400_000)
vals = [words[i] for i in ids]
chunk = writer.write_column_chunk(abi.BYTE_ARRAY, vals, abi.RLE_DICTIONARY, page_rows=5000)
batch = writer.build_batch([chunk])
lens = np.array([len(v) for v in vals], dtype=np.int64)
exp_off = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)]))
exp_data = torch.from_numpy(np.frombuffer(b"".join(vals), dtype=np.uint8).copy())
dec = D.Decoder(0, poison=0xA5)
dbatch = dec.upload(batch)
cols = dec.alloc_columns(batch)
plan = dec.plan(dbatch, cols)
def same(c):
    off = c.offsets().cpu()
    return bool(torch.equal(off, exp_off)) and bool(torch.equal(c.binary_data[: int(off[-1])].cpu(), exp_data))
out = {}
plan.launch()
rc, st = plan.sync()
out["first"] = {"rc": rc, "fallbacks": plan.timeout_fallbacks, "equal": same(cols[0])}
cols[0].binary_data.fill_(0xA5)
cols[0].values.fill_(0xA5)
plan.launch()
rc, st = plan.sync()
out["second"] = {"rc": rc, "fallbacks": plan.timeout_fallbacks, "equal": same(cols[0])}
plan.close()
dec.close()
print("RESULT " + json.dumps(out))
"""


@pytest.mark.gpu
def test_timed_out_dictionary_direct_launch_is_rerun_split_and_bit_exact(tmp_path):
    """A dictionary-direct BYTE_ARRAY column (k_dict_fused_dd: walk + compact ids + chunk byte sums in
    one launch): the injected walker delay times the launch out and pqg_sync re-runs it in split mode
    (k_dict_runs<4> + k_dict_tiles_dd, then k_dd_bases / k_dd_str); offsets and bytes are bit-exact."""
    assert os.path.exists(INJECT_LIB), "build() makes the fault-injection library"
    script = tmp_path / "child_dd.py"
    script.write_text(CHILD_DD)
    env = dict(os.environ, PQGPU_LIB=INJECT_LIB)
    r = subprocess.run([sys.executable, str(script), REPO], env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1]
    res = json.loads(line[7:])
    f = res["first"]
    assert f["rc"] == 0 and f["equal"], res
    assert f["fallbacks"] == 1, res
    s = res["second"]
    assert s["rc"] == 0 and s["equal"] and s["fallbacks"] == 1, res
