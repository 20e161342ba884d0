import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

CKPT = os.path.join(ROOT, "assets", "hf_predict_model.pkl")


def pytest_configure(config):
    # host mirrors run many tiny tensor ops: with 8 intra-op threads this container's OpenMP pool
    # costs ~10 ms per op (measured: torch.round on 2,400 doubles 10 ms vs 10 µs single-threaded)
    import torch
    torch.set_num_threads(1)
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running")


def _gpu_ok():
    import torch
    return torch.cuda.is_available()


def pytest_collection_modifyitems(config, items):
    if _gpu_ok():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def ckpt_path():
    return CKPT


@pytest.fixture(scope="session")
def dev():
    import torch
    from hfens import ops
    ops.ext()  # fail loudly if the HIP extension is missing on a GPU box
    return torch.device("cuda:0")
