"""Load tests/golden fixtures: column chunks (framing.read_column_chunk) + expected values."""
import json
import os

import numpy as np

from pqgpu import abi, framing, writer

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def chunk_cases():
    m = manifest()
    for name, v in m.items():
        for c in v["chunks"]:
            yield name, c


def load_chunk(name, c):
    buf = np.fromfile(os.path.join(GOLDEN, name + ".parquet"), dtype=np.uint8)
    ptype = framing.TYPE_BY_NAME[c["physical_type"]]
    ch = framing.read_column_chunk(buf, c["start"], c["length"], ptype, max_def=c["max_def"], max_rep=c["max_rep"],
                                   type_length=c["type_length"], num_values=c["num_values"])
    exp = np.load(os.path.join(GOLDEN, name + ".npz"))
    key = c["key"]
    if ptype == abi.BYTE_ARRAY:
        lens = exp[key + "_lens"]
        data = exp[key + "_bytes"].tobytes()
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        expected = [data[offs[i]:offs[i + 1]] for i in range(len(lens))]
    elif ptype in (abi.FIXED_LEN_BYTE_ARRAY, abi.INT96):
        w = abi.elem_width(ptype, c["type_length"])
        expected = np.ascontiguousarray(exp[key]).reshape(-1, w).view((np.void, w)).reshape(-1)
    else:
        expected = exp[key]
    ch.values = expected
    return ch, expected


def batch_of(ch):
    b = writer.build_batch([ch])
    return b
