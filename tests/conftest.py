import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "nvidia-jetson-workload_amd")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(autouse=True)
def _exact_numerics(monkeypatch):
    """Every test runs the fused kernels in exact numerics (bit-for-bit with the reference)
    unless it asks otherwise: fp64 simulations default to fast numerics (ws_hip.h), which
    tests/test_gpu_numerics.py covers against its tolerance."""
    monkeypatch.setenv("WS_NUMERICS", "exact")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running full-size case")


class Golden:
    """Reference outputs (tests/golden/gen_golden.py) for one precision."""

    def __init__(self, variant):
        self.variant = variant
        self.z = np.load(os.path.join(GOLDEN, f"ref_small_{variant}.npz"))
        self.meta = json.loads(self.z["__meta__"].tobytes().decode())

    def snap(self, case, snap):
        fields = ("u", "v", "h", "p", "t", "q", "vort")
        out = {k: self.z[f"{case}/{snap}/{k}"] for k in fields}
        out.update(self.meta[case][snap])
        return out

    def cases(self, prefix):
        return sorted(c for c in self.meta if c.startswith(prefix))


_GOLD = {}


def golden(variant):
    if variant not in _GOLD:
        _GOLD[variant] = Golden(variant)
    return _GOLD[variant]


@pytest.fixture(params=["f32", "f64"])
def gold(request):
    return golden(request.param)


def large_digests():
    with open(os.path.join(GOLDEN, "ref_large.json")) as f:
        return json.load(f)
