import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "lipreading-video-generation_amd")
DROPIN = os.path.join(PKG, "video-generation", "diffusion")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvdiff.so)")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


_cache = {}


def record_metric(**kw):
    """Append one JSON line of measured parity numbers to $VDIFF_TEST_METRICS, when set
    (tools/final_round.sh / tools/gpu_check.sh): pytest -q drops the tests' prints, so the
    measured errors of the parity tests are kept in a file that is committed under profiles/."""
    import json
    path = os.environ.get("VDIFF_TEST_METRICS")
    if path:
        with open(path, "a") as f:
            f.write(json.dumps(kw, sort_keys=True) + "\n")


def golden(name):
    if name not in _cache:
        with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
            _cache[name] = {k: torch.from_numpy(z[k].copy()) for k in z.files}
    return _cache[name]


@pytest.fixture
def gold():
    return golden
