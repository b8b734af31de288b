import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run via gpurun")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def native_mod():
    from kubernetes_machine_learning_server_amd.ops import native
    return native.load()


@pytest.fixture(scope="session")
def gpu_mod(native_mod):
    if not native_mod.gpu_available():
        pytest.fail("GPU test selected but no HIP device is visible (native GPU path must run)")
    return native_mod
