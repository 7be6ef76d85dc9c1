import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

SCENES = os.path.join(ROOT, "scenes")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernel through the C ABI)")
    config.addinivalue_line("markers", "slow: long CPU-side run")


def scene_path(name: str) -> str:
    return os.path.join(SCENES, name if name.endswith(".json") else name + ".json")


@pytest.fixture(scope="session")
def have_gpu():
    import torch  # noqa: F401  (binds the process to torch's HIP runtime before librt2 loads)
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True
