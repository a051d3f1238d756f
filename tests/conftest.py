"""Shared test plumbing. Markers: `gpu` (needs an MI355X + the built HIP library), `slow`."""
import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
GOLDEN = ROOT / "tests" / "golden"
PKG_ROOT = ROOT / "yolo-ad-refine_amd"
for p in (str(PKG_ROOT), str(ROOT / "oracle"), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X and the built libadr_hip.so")
    config.addinivalue_line("markers", "slow: long-running")


def golden(name):
    return np.load(GOLDEN / f"{name}.npz", allow_pickle=False)


def manifest():
    return json.loads((GOLDEN / "MANIFEST.json").read_text())


def state_dict_spec(tag="701"):
    return [(k, tuple(s), dt) for k, s, dt in manifest()[f"state_dict_{tag}"]]


@pytest.fixture(scope="session")
def cpu_threads():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    return torch.get_num_threads()
