import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librav1d_amd.so on the device)")


@pytest.fixture(scope="session")
def oracle():
    from tests.oracle_lib import load_oracle
    return load_oracle()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from rav1d_amd.frame import Context
    return Context(0)
