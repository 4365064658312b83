import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "f5-tts_amd"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: long CPU case")


@pytest.fixture(scope="session")
def torch_threads():
    import torch

    torch.set_num_threads(min(8, os.cpu_count() or 1))
    return torch.get_num_threads()
