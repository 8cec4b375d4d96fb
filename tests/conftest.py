"""Test configuration: import paths, the `gpu` marker and shared fixtures.

`-m "not gpu"` (the CPU suite) covers the oracle against the golden vectors, the native
host code (operand builder), the C-ABI exports and the multi-rank logic over gloo.
`-m gpu` holds the parity tests proper: the HIP kernels through the C ABI against the
oracle and the goldens.
"""
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "gnn-recommendations_amd"
GOLDEN = ROOT / "tests" / "golden"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libgnnrec.so")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


def load_golden(name):
    with np.load(GOLDEN / f"{name}.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_csr(name):
    """(row_ptr, col, val, n_users, n_items) of a reference-built normalised graph."""
    g = load_golden(f"graph_{name}")
    N = int(g["n_users"]) + int(g["n_items"])
    rp = np.zeros(N + 1, np.int64)
    np.add.at(rp, g["row"] + 1, 1)
    rp = np.cumsum(rp)
    return rp, g["col"].astype(np.int32), g["val"], int(g["n_users"]), int(g["n_items"])


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU visible")
    return torch.device("cuda", 0)
