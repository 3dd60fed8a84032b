import os
import sys
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def pytest_collection_modifyitems(config, items):
    # GPU tests never silently pass on a CPU box: they are skipped loudly when
    # no device is present, and fail (not skip) when the device is there but
    # the native library is not.
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def native():
    from vsr_amd import _native
    return _native.load(build_if_missing=True)


def load_golden(name):
    return torch.load(GOLDEN / f"{name}.pt", weights_only=True)
