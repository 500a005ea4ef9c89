import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and libhop_amd.so")
    config.addinivalue_line("markers", "devbuild: an A/B schedule of the developer library "
                            "(HOP_DEV_BUILD=1, HOP_LIB=...libhop_amd_dev.so); deselected otherwise")


def _dev_library():
    try:
        from time_opt_ilqr_amd import _lib
        return _lib.dev_build()
    except Exception:  # library not built or not loadable here
        return False


def pytest_collection_modifyitems(config, items):
    """A/B schedules exist only in the developer library: with the product library
    their cases are deselected (they test nothing the product runs)."""
    marked = [it for it in items if it.get_closest_marker("devbuild")]
    if not marked or _dev_library():
        return
    keep = [it for it in items if not it.get_closest_marker("devbuild")]
    config.hook.pytest_deselected(items=marked)
    items[:] = keep


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    from time_opt_ilqr_amd import build
    build.build(verbose=False)
    return torch.device("cuda", 0)
