"""pqg_unpack_runs over many runs in one call (ParquetReadRouter.read / BytePacker.unpack8Values,
parquet-plugins/.../ParquetReadRouter.java:57-66, ByteBasedBitPackingGenerator.java:258-308): runs of
different lengths at arbitrary byte offsets, every width 0..32, bit-exact with the oracle's
unpack8Values restatement (oracle/pqref.c, pinned to TestBitPacking / the generator's vectors)."""
import ctypes as C

import numpy as np
import pytest
import torch

from oracle import pqref
from pqgpu import native

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("w", list(range(0, 33)))
def test_many_runs_one_call(decoder, w):
    rng = np.random.default_rng(w + 3)
    n_runs = 300
    counts = (rng.integers(1, 64, size=n_runs) * 8).astype(np.uint32)     # whole groups of 8
    nbytes = counts.astype(np.int64) * w // 8
    gaps = rng.integers(0, 5, size=n_runs)                                  # runs at any byte offset
    in_off = np.zeros(n_runs, dtype=np.uint64)
    pos = 0
    for r in range(n_runs):
        pos += int(gaps[r])
        in_off[r] = pos
        pos += int(nbytes[r])
    data = rng.integers(0, 256, size=pos + 16, dtype=np.uint8)
    out_off = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(np.uint64)
    expect = np.zeros(int(counts.sum()), dtype=np.int32)
    for r in range(n_runs):
        o, b = int(out_off[r]), int(in_off[r])
        for g in range(int(counts[r]) // 8):
            expect[o + 8 * g: o + 8 * g + 8] = pqref.unpack8_int(w, data[b + g * w: b + g * w + max(w, 1)].tobytes())
    dev = decoder.device
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    d_in, d_io, d_cnt, d_oo = t(data), t(in_off.view(np.int64)), t(counts.view(np.int32)), t(out_off.view(np.int64))
    d_out = torch.full((int(counts.sum()),), -7, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    rc = native.lib().pqg_unpack_runs(decoder.ctx, w, C.c_void_p(d_in.data_ptr()), C.c_void_p(d_io.data_ptr()),
                                      C.c_void_p(d_cnt.data_ptr()), C.c_void_p(d_oo.data_ptr()),
                                      C.c_void_p(d_out.data_ptr()), n_runs)
    assert rc == 0
    torch.cuda.synchronize()  # the kernel ran on the decoder's stream
    assert np.array_equal(d_out.cpu().numpy(), expect)
