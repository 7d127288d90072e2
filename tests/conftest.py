import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "parquet-mr_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


def _gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def decoder():
    from pqgpu import decoder as D
    dec = D.Decoder(0, poison=0xA5)  # unwritten output elements show up as 0xA5A5...
    yield dec
    dec.close()


@pytest.fixture(params=["wave_per_page", "lane_per_page"])
def level_kernel(decoder, request):
    """Level sections through both level kernels: k_levels (one wave per page, the default below
    PQG_DISPATCH_LEVELS_LANE_MIN pages) and k_levels_lane (one lane per page; forced with 0)."""
    from pqgpu import abi
    if request.param == "lane_per_page":
        decoder.set_dispatch(abi.DISPATCH_LEVELS_LANE_MIN, 0)
    yield request.param
    decoder.set_dispatch(abi.DISPATCH_LEVELS_LANE_MIN, 2048)
