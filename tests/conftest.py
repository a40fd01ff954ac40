import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libbpftime_amd.so on the device)")


@pytest.fixture(scope="session")
def gpu():
    """Skip-free GPU guard: gpu tests must run on a box with a device."""
    from bpftime_amd._lib import lib
    n = lib().bpftime_amd_device_count()
    assert n > 0, "no HIP device visible"
    return n


@pytest.fixture()
def fresh_oracle():
    from oracle import pyoracle as po
    po.reset()
    po.set_ncpu(1)
    po.set_cpu(0)
    yield po
    po.reset()


@pytest.fixture()
def fresh_runtime(gpu):
    from bpftime_amd import vm
    vm.reset_runtime()
    vm.set_ncpu(64)
    yield vm
    vm.reset_runtime()
