import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "jabd-joint-attention-based-detector-for-small-face-detection_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")

# spawned test workers import jabd_amd too
os.environ["PYTHONPATH"] = os.pathsep.join(
    [PKG, ROOT] + [p for p in os.environ.get("PYTHONPATH", "").split(os.pathsep) if p])
