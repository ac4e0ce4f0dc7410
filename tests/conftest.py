import glob
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "d2d-ppo_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")


def load_params(z):
    """Rebuild the constructor kwargs stored in a golden env fixture."""
    raw = json.loads(str(z["params_json"]))
    out = {}
    for k, v in raw.items():
        if isinstance(v, dict) and "__nd__" in v:
            out[k] = np.array(v["__nd__"], dtype=v["dtype"])
        else:
            out[k] = v
    return out


def env_fixture_names():
    return sorted(os.path.basename(p)[4:-4] for p in glob.glob(os.path.join(GOLDEN, "env_*.npz")))


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
