"""Inputs beyond the round-3 caps, against the reference's own renders.

Goldens: tests/golden/render_r4.npz + golden_r4.json (tools/gen_golden_r4.py,
rendered by the reference itself):

* breakpoint lanes of 40 and 200 points on all four lanes (MS:452-482, 602-605,
  634-637; the UI's lane fields are free text, MS:1070-1073): variable-length
  lanes in a per-batch breakpoint bank (include/msgpu.h);
* 300 resonator modes (MS:369-384), 300 wavelet atoms (MS:317-331), 300
  waveguide lines (MS:386-402) and 300 locked peaks (MS:130-148), reachable
  through preset JSON: the float64 chain draws and applies them 256 at a time;
* CLIP192: ER + IR taps longer than the output at 192 kHz.

Tolerance: 1e-5 RMS over the (out_n, 2) buffer (north star).
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-5
CASES = ["LANES40", "LANES200", "RES300", "WAV300", "WG300", "PL300", "CLIP192"]


@pytest.fixture(scope="module")
def r4():
    with open(os.path.join(GOLDEN, "golden_r4.json")) as fh:
        info = json.load(fh)
    return info, np.load(os.path.join(GOLDEN, "render_r4.npz"))


def params_of(info, irs, name):
    import msgpu
    p = dict(info["params"][name])
    ir = p.pop("_ir", None)
    p = msgpu.merged(p)
    p["_ir_audio"] = irs[ir] if ir else None
    p["_img_gray"] = None
    return p


def rms(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    return float(np.sqrt(np.mean((a - b) ** 2)))


@pytest.mark.parametrize("name", CASES)
def test_uncapped_inputs_match_reference(r4, irs, name):
    import msgpu
    info, arrays = r4
    p = params_of(info, irs, name)
    audio, meta = msgpu.render(p)
    err = rms(audio, arrays[f"{name}_audio"])
    print(f"{name}: rms err {err:.3e}")
    assert meta["design_sr_base"] == info["summaries"][name]["design_sr_base"]
    assert err <= RMS_TOL


def test_uncapped_inputs_as_one_batch(r4, irs):
    """All cases in one device batch (lanes of several lengths in one bank)."""
    import msgpu
    info, arrays = r4
    outs = msgpu.render_batch([params_of(info, irs, n) for n in CASES])
    for name, a in zip(CASES, outs):
        assert rms(a, arrays[f"{name}_audio"]) <= RMS_TOL, name
