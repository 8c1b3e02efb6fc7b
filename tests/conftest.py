import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("oracle", "proxmox-backup_amd"):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: large-size GPU properties")


@pytest.fixture(scope="session")
def oracle():
    import oracle as o
    o.lib()
    return o


@pytest.fixture(scope="session")
def pbschunk():
    import pbschunk as p
    return p


@pytest.fixture(scope="session")
def gpu(pbschunk):
    if pbschunk.device_count() <= 0:
        pytest.fail("-m gpu test without a visible HIP device")
    return pbschunk
