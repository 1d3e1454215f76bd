"""The Python examples of README.md and INTEGRATION.md §1 run as written (GPU)."""
import os
import re

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ws = pytest.importorskip("weather_sim")
if not ws.is_cuda_available():  # pragma: no cover
    pytest.skip("no HIP device", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _python_blocks(doc, section=None):
    text = open(os.path.join(ROOT, doc)).read()
    if section:
        start = text.index(section)
        end = text.find("\n## ", start + 1)
        text = text[start:end if end > 0 else None]
    return re.findall(r"```python\n(.*?)```", text, re.S)


@pytest.mark.parametrize("doc,section", [("README.md", None), ("INTEGRATION.md", "## 1.")])
def test_doc_example_runs(doc, section, monkeypatch):
    monkeypatch.chdir(ROOT)
    blocks = [b for b in _python_blocks(doc, section) if "WeatherSimulationWrapper(" in b]
    assert blocks, f"no wrapper example in {doc}"
    env = {}
    exec(compile(blocks[0], f"{doc} example", "exec"), env)
    u, v = env["u"], env["v"]
    sim = env["sim"]
    W, H = sim.config.grid_width, sim.config.grid_height
    assert u.shape == v.shape == (H, W)
    assert np.isfinite(u).all() and np.isfinite(v).all()
    assert sim.simulation.get_current_step() == 100
