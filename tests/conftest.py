import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def nv():
    from allreduce_over_mpi_amd import _native

    _native.lib()  # builds libflexar.so in-tree if needed
    return _native


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from allreduce_over_mpi_amd import _native

    _native.lib()
    return torch.device("cuda", 0)
