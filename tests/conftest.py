import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    for m in (
        "gpu: needs a real MI355X (runs the HIP kernels)",
        "multigpu: needs >1 GPU",
        "slow: long-running",
        "pre_merge: fast CPU checks",
    ):
        config.addinivalue_line("markers", m)


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
