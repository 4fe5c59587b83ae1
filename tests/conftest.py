"""Test configuration.  `-m "not gpu"` runs on CPU (oracle vs golden vectors, host logic,
C-ABI load/export checks, gloo multi-process); `-m gpu` runs the HIP parity tests on MI355X."""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

GOLDEN = Path(__file__).resolve().parent / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device); runs the HIP kernels")


def pytest_sessionstart(session):
    """Refuse to test a stale prebuilt libeggroll.so: its source stamp (written by build_ext) must equal
    the digest of csrc/* + include/eggroll.h in this tree (content, not mtime — snapshots copied to a
    GPU box keep bytes, not timestamps)."""
    from hyperscalees_t2i_amd import _lib
    if _lib.LIB_PATH.exists() and not os.environ.get("EGGROLL_LIB"):
        try:
            _lib.check_fresh()
        except _lib.EggrollError as e:
            pytest.exit(f"libeggroll.so is stale: {e}", returncode=3)


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(GOLDEN / name, allow_pickle=False)
    return load


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no ROCm device is visible")
    return torch.device("cuda:0")
