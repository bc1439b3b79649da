import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (gfx950) GPU and the built HIP extension')


@pytest.fixture(scope='session')
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from mx_rcnn_amd.ops import need_ext
    need_ext()  # a GPU box must have the extension: fail loudly, never fall back
    return torch.device('cuda', 0)


@pytest.fixture(autouse=True)
def _reset_config():
    from mx_rcnn_amd import config as cfgmod
    snap = cfgmod.snapshot()
    yield
    cfgmod.restore(snap)
