import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


@pytest.fixture(scope="session")
def engine():
    # torch's HIP runtime must open the device before the engine's (ROCm) runtime does; with the
    # opposite order torch reports "No HIP GPUs are available" in the same process
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()
    from sda_amd import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O
