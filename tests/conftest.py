import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "multigpu: needs >= 2 GPUs on one node")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        have_gpu = torch.cuda.is_available()
        ngpu = torch.cuda.device_count() if have_gpu else 0
    except Exception:  # noqa: BLE001
        have_gpu, ngpu = False, 0
    skip_gpu = pytest.mark.skip(reason="no GPU on this host")
    skip_multi = pytest.mark.skip(reason="needs >= 2 GPUs: unverified on a 1-GPU host")
    for item in items:
        if "gpu" in item.keywords and not have_gpu:
            item.add_marker(skip_gpu)
        if "multigpu" in item.keywords and ngpu < 2:
            item.add_marker(skip_multi)
