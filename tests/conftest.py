"""Shared test setup: import paths, the ``gpu`` marker, golden fixture loaders."""
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (os.path.join(REPO, "audio-suite_amd"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libmsgpu.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def funcs():
    return np.load(os.path.join(GOLDEN, "funcs.npz"))


@pytest.fixture(scope="session")
def full_renders():
    return np.load(os.path.join(GOLDEN, "render_full.npz"))


@pytest.fixture(scope="session")
def large_renders():
    return np.load(os.path.join(GOLDEN, "render_large.npz"))


@pytest.fixture(scope="session")
def irs():
    z = np.load(os.path.join(GOLDEN, "irs.npz"))
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden_info():
    with open(os.path.join(GOLDEN, "golden_info.json")) as fh:
        return json.load(fh)


@pytest.fixture(scope="session")
def extra_renders():
    return np.load(os.path.join(GOLDEN, "render_extra.npz"))


@pytest.fixture(scope="session")
def golden_extra():
    with open(os.path.join(GOLDEN, "golden_extra.json")) as fh:
        return json.load(fh)


def extra_params(golden_extra, irs, name):
    """The params dict of a render_extra.npz case (tools/gen_golden_r3.py)."""
    import msgpu
    if name.startswith("H48_"):
        return msgpu.config_params("H48", seed=int(name.split("_")[1]), irs=irs)
    p = dict(golden_extra["params"][name])
    ir = p.pop("_ir", None)
    p = msgpu.merged(p)
    p["_ir_audio"] = irs[ir] if ir else None
    p["_img_gray"] = None
    return p
