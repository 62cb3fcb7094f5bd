import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible (run -m 'not gpu' on CPU hosts)")
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _repo_cwd(monkeypatch):
    """Fixture paths (tests/golden/...) are repo-relative: run every test from the repository root."""
    monkeypatch.chdir(ROOT)
