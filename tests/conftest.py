"""Shared test setup: import paths, the `gpu` marker, fixture loaders."""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "yieldfactormodels.jl_amd"
GOLDEN = Path(__file__).resolve().parent / "golden"
for p in (str(PKG), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libyfm_hip.so on a HIP device)")


def load_golden(name: str) -> dict:
    with np.load(GOLDEN / f"{name}.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


GOLDEN_NAMES = sorted(p.stem for p in GOLDEN.glob("*.npz"))


@pytest.fixture(scope="session")
def engine():
    import torch  # noqa: F401  (bind libyfm_hip to torch's HIP runtime when both are loaded)
    from yfm_amd import get_engine
    return get_engine(0)
