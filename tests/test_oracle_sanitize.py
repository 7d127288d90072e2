"""The oracle (oracle/pqref.c) under AddressSanitizer + UndefinedBehaviorSanitizer (host only; SURVEY
§5): a driver executable (oracle/sanitize_main.c) built with -fsanitize=address,undefined
-fno-sanitize-recover=all decodes every golden fixture chunk, writer-made pages of every encoding,
and deterministic mutations of them (flipped bytes, shortened pages, lying headers) into
exactly-sized heap outputs. Any out-of-bounds access or undefined behaviour aborts the run."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import fixtures
from pqgpu import abi
from tools.synth import writer

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(REPO, "oracle")


def serialize(batch, path, binary_capacity=None):
    cols = (abi.ColumnDesc * max(1, len(batch.columns)))()
    for i, cd in enumerate(batch.columns):
        for k, v in cd.items():
            setattr(cols[i], k, v)
        if cd["physical_type"] == abi.BYTE_ARRAY:
            cols[i].binary_capacity = binary_capacity if binary_capacity is not None else 4 * len(batch.data) + 4096
    pages = np.ascontiguousarray(batch.pages)
    data = batch.data.tobytes()
    with open(path, "wb") as f:
        f.write(b"PQGB" + np.uint32(len(batch.columns)).tobytes() + np.uint32(len(pages)).tobytes() +
                np.uint64(len(data)).tobytes())
        f.write(bytes(cols)[: C.sizeof(abi.ColumnDesc) * len(batch.columns)])
        f.write(pages.tobytes())
        f.write(data)


def base_batches():
    out = []
    for name, c in fixtures.chunk_cases():
        ch, _ = fixtures.load_chunk(name, c)
        out.append(fixtures.batch_of(ch))
    rng = np.random.default_rng(11)
    n = 3000
    dl = (rng.random(n) > 0.2).astype(np.uint8)
    k = int(dl.sum())
    for ver in (1, 2):
        for pt, enc in [(abi.INT64, abi.RLE_DICTIONARY), (abi.INT32, abi.DELTA_BINARY_PACKED),
                        (abi.INT64, abi.DELTA_BINARY_PACKED), (abi.DOUBLE, abi.PLAIN), (abi.FLOAT, abi.BYTE_STREAM_SPLIT),
                        (abi.BOOLEAN, abi.PLAIN), (abi.BOOLEAN, abi.RLE)]:
            if pt == abi.BOOLEAN:
                v = rng.integers(0, 2, size=k).astype(np.uint8)
            elif pt in (abi.DOUBLE, abi.FLOAT):
                v = rng.standard_normal(k).astype(abi.numpy_dtype(pt))
            else:
                v = rng.integers(-1000, 1000, size=k).astype(abi.numpy_dtype(pt))
            out.append(writer.build_batch([writer.write_column_chunk(pt, v, enc, def_levels=dl, max_def=1, version=ver,
                                                                     page_rows=700)]))
        for enc in (abi.PLAIN, abi.RLE_DICTIONARY, abi.DELTA_LENGTH_BYTE_ARRAY, abi.DELTA_BYTE_ARRAY):
            v = writer.BinaryValues.random(k, 0, 20, seed=ver)
            out.append(writer.build_batch([writer.write_column_chunk(abi.BYTE_ARRAY, list(v), enc, def_levels=dl,
                                                                     max_def=1, version=ver, page_rows=700)]))
    return out


def mutations(batch, rng, n):
    """Deterministic corruptions: flipped bytes inside page bodies, pages that claim fewer bytes /
    more values than they hold, a dictionary that claims fewer entries."""
    import copy
    res = []
    for _ in range(n):
        b = copy.copy(batch)
        b.data = batch.data.copy()
        b.pages = batch.pages.copy()
        b.columns = [dict(c) for c in batch.columns]
        kind = rng.integers(0, 4)
        if len(b.pages) == 0:
            break
        p = int(rng.integers(0, len(b.pages)))
        off, size = int(b.pages["offset"][p]), int(b.pages["size"][p])
        if kind == 0 and size:
            for _ in range(int(rng.integers(1, 6))):
                b.data[off + int(rng.integers(0, size))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif kind == 1 and size:
            b.pages["size"][p] = int(rng.integers(0, size))
        elif kind == 2:
            b.pages["num_values"][p] = int(b.pages["num_values"][p]) + int(rng.integers(1, 100))
        elif kind == 3 and b.columns[0]["dict_offset"] >= 0:
            b.columns[0]["dict_num_values"] = int(rng.integers(0, max(1, b.columns[0]["dict_num_values"])))
        res.append(b)
    return res


def test_oracle_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "sanitize_main")
    subprocess.run(["gcc", "-std=c11", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-I", ORACLE, "-I", os.path.join(REPO, "include"),
                    os.path.join(ORACLE, "sanitize_main.c"), os.path.join(ORACLE, "pqref.c"), "-o", exe], check=True)
    rng = np.random.default_rng(5)
    files = []
    for i, b in enumerate(base_batches()):
        for j, m in enumerate([b] + mutations(b, rng, 6)):
            path = str(tmp_path / f"case_{i}_{j}.bin")
            serialize(m, path)
            files.append(path)
        if any(c["physical_type"] == abi.BYTE_ARRAY for c in b.columns):
            path = str(tmp_path / f"case_{i}_short.bin")  # binary capacity too small: must stop, not overflow
            serialize(b, path, binary_capacity=7)
            files.append(path)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([exe] + files, capture_output=True, text=True, env=env, timeout=600)
    assert out.returncode == 0, out.stderr[-4000:]
    lines = out.stdout.splitlines()
    assert len(lines) == len(files)
    codes = [int(ln.rsplit("rc=", 1)[1]) for ln in lines]
    assert codes.count(0) >= len(base_batches())      # the unmutated cases decode
    assert sum(c != 0 for c in codes) >= len(files) // 4  # and the corruptions are reported, not crashed on
