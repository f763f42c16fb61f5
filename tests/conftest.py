import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle_lib():
    from tests.oracle_lib import load_oracle
    return load_oracle()


@pytest.fixture(scope="session")
def gx_lib():
    from sidecar_amd.abi import load_product
    return load_product()
