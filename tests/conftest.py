import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Deterministic convolution tilings in the test processes: the persistent
# table (the benched tilings at the bench shapes), the cost model on a miss --
# never a per-run timing choice, whose summation order could differ from run
# to run (include/hcunet.h, hcu_tuning_set_mode).  Read when the library
# first plans; a test that needs another mode sets it itself.
os.environ.setdefault('HCU_BCONV_TUNE', '1')


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) device")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm device in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
