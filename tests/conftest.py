import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP kernels, RCCL); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def C():
    from mpi_cuda_amd._native import load

    return load()


@pytest.fixture(scope="session")
def gpu(C):
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible (the HIP path must run, no fallback)")
    return C
