"""Debug: the harness's call sequence through ctypes on a context with the LIBRARY's own stream."""
import ctypes as C
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "parquet-mr_amd"), os.path.join(REPO, "tests"), REPO]
import fixtures  # noqa: E402
from pqgpu import abi, framing, native  # noqa: E402

name, key = sys.argv[1], sys.argv[2]
own = sys.argv[3] == "own"
for n, c in fixtures.chunk_cases():
    if n == name and c["key"] == key:
        break
ch, exp = fixtures.load_chunk(name, c)
buf = np.fromfile(os.path.join(fixtures.GOLDEN, name + ".parquet"), dtype=np.uint8).tobytes()
raw = np.frombuffer(buf[c["start"]: c["start"] + c["length"]], dtype=np.uint8).copy()
rc, st, hdrs = framing.frame_chunk_native(raw.tobytes(), c["num_values"])
L = native.lib()
arr = (abi.PageHeader * len(hdrs))(*hdrs)
col = abi.ColumnDesc()
col.dict_offset = -1
pages = (abi.PageDesc * len(hdrs))()
nn = C.c_int(0)
L.pqg_pages_from_headers(C.addressof(arr), len(hdrs), 0, 0, C.byref(col), C.addressof(pages), len(hdrs), C.byref(nn), C.byref(st))
col.physical_type = ch.physical_type
ctx = C.c_void_p()
if own:
    L.pqg_ctx_create(0, None, C.byref(ctx))
else:
    import torch
    s = torch.cuda.Stream(torch.device("cuda", 0))
    L.pqg_ctx_create(0, C.c_void_p(s.cuda_stream), C.byref(ctx))
slots = sum(pages[k].num_values for k in range(nn.value))
offs = np.zeros(slots + 1, dtype=np.int64)
counts = np.zeros(nn.value + 1, dtype=np.uint32)
for cap in (2864, 36064, 36064):
    bd = np.zeros(cap, dtype=np.uint8)
    col.values = offs.ctypes.data
    col.values_capacity = slots + 1
    col.levels_capacity = slots
    col.binary_data = bd.ctypes.data
    col.binary_capacity = cap
    st = abi.Status()
    rc = L.pqg_decode_host(ctx, raw.ctypes.data, raw.size, C.byref(col), 1, C.addressof(pages), nn.value,
                           counts.ctypes.data, C.byref(st))
    n = int(col.values_written)
    vals = [bd[offs[i]:offs[i + 1]].tobytes() for i in range(n)] if rc == 0 else []
    bad = [i for i in range(len(vals)) if vals[i] != bytes(exp[i])]
    print("own" if own else "torch", "cap", cap, "rc", rc, st.message[:50], "n", n, "bad", len(bad), bad[:4], offs[-3:])
L.pqg_ctx_destroy(ctx)
