import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def gpu_worker_factory():
    """GPU tests fail loudly (no skip, no fallback) when the HIP library or device is missing."""
    from upe_amd import gpu

    n = gpu.device_count()
    assert n and n > 0, f"no GPU visible to libupe_gpu.so ({gpu.LIB.upe_gpu_last_error()!r})"

    def make(capacity=1024, device=0):
        return gpu.GpuWorker(device, capacity)

    return make
