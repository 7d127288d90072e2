"""Host check of the XCD-aware workgroup order used by the expansion kernels
(pqg::xcd_order, parquet-mr_amd/csrc/pqgpu_device.h): a bijection with one contiguous run per XCD."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not present")
def test_xcd_order_bijection(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    exe = tmp_path / "xcd_order"
    subprocess.run([hipcc, "-O1", "-std=c++17", "-I", os.path.join(REPO, "parquet-mr_amd", "csrc"),
                    os.path.join(REPO, "tests", "c", "xcd_order.cpp"), "-o", str(exe)], check=True,
                   capture_output=True, timeout=300)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.strip() == "ok", out.stdout + out.stderr
