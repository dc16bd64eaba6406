import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# spark.executor.instances defaults to "auto" (every visible GPU): a test session built from
# SessionConf() must stay in-process even on a multi-GPU box; pool tests set it explicitly
os.environ.setdefault("O3S_CONF_SPARK__EXECUTOR__INSTANCES", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (ROCm GPU); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


HAS_GPU = _has_gpu()


def pytest_collection_modifyitems(config, items):
    if HAS_GPU:
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def gpu():
    import torch
    return torch.device("cuda", 0)
