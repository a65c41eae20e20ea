import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("", "volumetric-renderer_amd", "oracle", "tools"):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    """Skip-free on the GPU box: a gpu-marked test without a device is an error, not a skip."""
    if not _has_gpu():
        pytest.fail("GPU test selected but no HIP device is visible")
    return 0


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the product library and the oracle once per session (no-op when up to date)."""
    import subprocess
    if os.path.exists("/root/reference") or not os.path.exists(
            os.path.join(ROOT, "volumetric-renderer_amd", "lib", "libvr_amd.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "volumetric-renderer_amd")], check=True)
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "oracle"], check=True)
