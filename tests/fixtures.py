"""Load tests/golden fixtures: column chunks (framing.read_column_chunk) + expected values."""
import json
import os

import numpy as np

from pqgpu import abi, framing
from tools.synth import writer

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
    # (pyarrow names the LZ4_RAW codec it writes "LZ4")
    codec = {"SNAPPY": writer.SNAPPY, "ZSTD": writer.ZSTD, "LZ4": writer.LZ4_RAW, "LZ4_RAW": writer.LZ4_RAW,
             "GZIP": writer.GZIP}.get(c.get("compression"), writer.UNCOMPRESSED)
    ch = framing.read_column_chunk(buf, c["start"], c["length"], ptype, max_def=c["max_def"], max_rep=c["max_rep"],
                                   type_length=c["type_length"], num_values=c["num_values"], codec=codec)
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


def is_compressed(ch):
    return ch.dict_codec != writer.UNCOMPRESSED or any(p.codec != writer.UNCOMPRESSED for p in ch.pages)


def decompressed_on_host(ch):
    """The chunk with every SNAPPY / ZSTD / LZ4_RAW / GZIP page decompressed by the ORACLE (test infrastructure)."""
    import copy

    from oracle import pqref
    unzs = {writer.ZSTD: pqref.zstd_decompress, writer.SNAPPY: pqref.snappy_decompress,
            writer.LZ4_RAW: pqref.lz4_raw_decompress, writer.GZIP: pqref.gzip_decompress}
    out = copy.deepcopy(ch)
    if out.dict_codec:
        unz = unzs[out.dict_codec]
        out.dict_page = unz(out.dict_page, out.dict_uncompressed_size)
        out.dict_codec = writer.UNCOMPRESSED
    for p in out.pages:
        if p.codec:
            lv = p.rl_byte_length + p.dl_byte_length if p.version == 2 else 0
            unz = unzs[p.codec]
            p.body = p.body[:lv] + unz(p.body[lv:], p.uncompressed_size - lv)
            p.codec = writer.UNCOMPRESSED
    return out


def batch_of(ch):
    """Host batch of a fixture chunk (compressed pages decompressed by the oracle)."""
    return writer.build_batch([decompressed_on_host(ch) if is_compressed(ch) else ch])
