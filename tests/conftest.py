import os
import sys

import pytest

# torch's own convolutions appear only as test-side references (fp32 autograd of the
# decoder at the training batch): MIOpen's immediate-mode heuristics instead of its
# per-shape benchmarking search, which takes minutes on the large shapes
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libtcam_hip.so")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
