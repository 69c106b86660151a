"""Shared test plumbing.

Markers: `gpu` = needs a ROCm GPU (MI355X) and the built librecsys_hip.so; everything else runs
on CPU. The parity tests compare the HIP path with the oracle (oracle/recsys_oracle.py, a numpy
restatement of the reference arithmetic) on the same seeded inputs.
"""
import importlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PKG_NAME = "recommendation-system-maang-nvidia-_amd"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running")


def pkg(sub=None):
    name = PKG_NAME if sub is None else f"{PKG_NAME}.{sub}"
    return importlib.import_module(name)


def oracle():
    return importlib.import_module("oracle.recsys_oracle")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU visible")
    pkg("_native").load()  # fail loudly if the extension is missing on a GPU box
    return torch.device("cuda")


def rel_err(a, b, floor=1.0):
    """max |a - b| / max(floor, max |b|): absolute error for O(1) values, relative to the
    tensor's scale for large ones (floor=0 makes it purely scale-relative)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if a.shape != b.shape:
        raise AssertionError(f"shape mismatch {a.shape} vs {b.shape}")
    if not a.size:
        return 0.0
    den = max(floor, float(np.max(np.abs(b))))
    if den == 0.0:
        den = 1.0
    return float(np.max(np.abs(a - b))) / den


def assert_close(a, b, tol=1e-4, what="", floor=1.0):
    e = rel_err(a, b, floor)
    assert e <= tol, f"{what}: max|a-b|/max({floor},|b|max) = {e:.3e} > {tol:.1e}"
