"""pytest setup: package path, the ``gpu`` marker, shared fixture helpers."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "physics-llm-inference_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm (MI355X) device and libpli_hip.so")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm device")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def built_lib():
    """Path of libpli_hip.so, building it in-tree if it is missing (hipcc
    cross-compiles gfx950 without a GPU)."""
    sys.path.insert(0, PKG)
    import build as pli_build  # physics-llm-inference_amd/build.py
    lib = os.path.join(PKG, "pli_hip", "libpli_hip.so")
    if not os.path.exists(lib):
        pli_build.build(verbose=False)
    return lib


def load_golden(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}
