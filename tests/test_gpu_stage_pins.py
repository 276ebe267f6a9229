"""The float64 chain at the input of the two ill-conditioned stages.

Seven shipped presets are held to the reference's own rounding spread over the
whole render (test_gpu_parity.py::test_all_shipped_presets, DESIGN.md section
2): the cepstral warp takes log(|X| + 1e-12) (MS:154) and the spectral imprint
re-imposes angle(X) (MS:580), both of which read float64 rounding noise in
band-limited bins.  These tests pin the device's float64 chain right BEFORE
those steps, where nothing is ill-conditioned: the last event's grain as the
reference's cepstral_warp / SpectralImprint.apply received it
(tests/golden/stage_pins.npz, tools/gen_stage_pins.py), to <= 1e-9 relative
RMS.  For the cepstral presets the library stops the chain before the warp
(MSGPU_G64_STOP=cep); the imprint input is meta["grain_last"] (the grain
before feedback and imprint, MS:729) of presets without event feedback or
cepstral warp (whose output it would inherit).
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-9


@pytest.fixture(scope="module")
def pins():
    return np.load(os.path.join(GOLDEN, "stage_pins.npz"))


def _preset(name, golden_info, irs, full_renders):
    import msgpu
    p = msgpu.merged(golden_info["preset_params"][name])
    p["out_dur_s"] = 0.5
    p["_ir_audio"] = irs["tiny_room_ir"]
    p["_img_gray"] = full_renders["image_gray"]
    return p


def _rel(a, b):
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(1e-300, np.sqrt(np.mean(b ** 2))))


@pytest.mark.parametrize("name", ["ghost_formants", "03_wavelet_ice_bloom", "wavelet_mist", "closed_curve_air",
                                  "drifting_mode_fragments", "corona_glass_fog"])
def test_cepstral_input(name, pins, golden_info, irs, full_renders, monkeypatch):
    import msgpu
    ref = pins[f"{name}_cep"]
    monkeypatch.setenv("MSGPU_G64_STOP", "cep")
    _, meta = msgpu.render(_preset(name, golden_info, irs, full_renders))
    g = meta["grain_last"]
    assert g is not None and g.dtype == np.float64 and g.shape == ref.shape
    err = _rel(g, ref)
    print(f"{name}: cepstral_warp input rel rms err {err:.3e}")
    assert err <= TOL


# corona_glass_fog's imprint input comes after its cepstral warp, so it carries
# that step's spread (5.7e-4 measured); its chain is pinned at the cepstral input
@pytest.mark.parametrize("name", ["soft_ellipse_memory"])
def test_imprint_input(name, pins, golden_info, irs, full_renders):
    import msgpu
    p = _preset(name, golden_info, irs, full_renders)
    assert not p["event_feedback_on"]
    ref = pins[f"{name}_imp"]
    _, meta = msgpu.render(p)
    g = meta["grain_last"]
    assert g is not None and g.shape == ref.shape
    err = _rel(g, ref)
    print(f"{name}: SpectralImprint.apply input rel rms err {err:.3e}")
    assert err <= TOL


def test_pins_cover_the_spread_presets():
    with open(os.path.join(GOLDEN, "render_spread.json")) as f:
        spread = json.load(f)["spread"]
    z = np.load(os.path.join(GOLDEN, "stage_pins.npz"))
    names = {k.rsplit("_", 1)[0] for k in z.files if k != "info"}
    held = {k for k, v in spread.items() if 1.5 * v > 1e-5}        # the presets held to the spread
    assert held <= names, held - names


# ---- every event (round 3): tests/golden/stage_pins_all.npz holds every call's input
@pytest.fixture(scope="module")
def pins_all():
    return np.load(os.path.join(GOLDEN, "stage_pins_all.npz"))


def _per_event(name, stage, golden_info, irs, full_renders, pins_all):
    """Device float64 grain of every event vs the reference's input to `stage` in
    the same call order; returns the relative errors."""
    import torch
    from msgpu.engine import default_engine
    from msgpu.pack import PackedBatch
    lens = pins_all[f"{name}_{stage}_lens"]
    data = pins_all[f"{name}_{stage}_data"]
    eng = default_engine(0)
    eng.render_packed(PackedBatch([_preset(name, golden_info, irs, full_renders)]))
    torch.cuda.synchronize(0)
    assert len(eng.last_events(0)) == len(lens), (name, len(eng.last_events(0)), len(lens))
    errs, at = [], 0
    for k, n in enumerate(lens):
        ref = data[at:at + n]
        at += n
        g = eng.last_grain64(0, k)
        assert g.shape == ref.shape, (name, k, g.shape, ref.shape)
        errs.append(_rel(g, ref))
    return errs


@pytest.mark.parametrize("name", ["ghost_formants", "03_wavelet_ice_bloom", "wavelet_mist", "closed_curve_air",
                                  "drifting_mode_fragments", "corona_glass_fog"])
def test_cepstral_input_every_event(name, pins_all, golden_info, irs, full_renders, monkeypatch):
    monkeypatch.setenv("MSGPU_G64_STOP", "cep")
    errs = _per_event(name, "cep", golden_info, irs, full_renders, pins_all)
    print(f"{name}: cepstral_warp inputs of {len(errs)} events, rel rms err max {max(errs):.3e} "
          f"median {float(np.median(errs)):.3e}: " + " ".join(f"{e:.1e}" for e in errs))
    assert max(errs) <= TOL


def test_imprint_input_every_event(pins_all, golden_info, irs, full_renders):
    name = "soft_ellipse_memory"
    errs = _per_event(name, "imp", golden_info, irs, full_renders, pins_all)
    print(f"{name}: SpectralImprint.apply inputs of {len(errs)} events, rel rms err max {max(errs):.3e}: "
          + " ".join(f"{e:.1e}" for e in errs))
    assert max(errs) <= TOL


def test_grain64_readback_bounds(golden_info, irs, full_renders):
    """msg_last_grain64 refuses event indices outside the preset's events and
    presets that are not on the float64 chain (RuntimeError), instead of reading
    another preset's record."""
    import torch
    import msgpu
    from msgpu.engine import default_engine
    from msgpu.pack import PackedBatch
    eng = default_engine(0)
    eng.render_packed(PackedBatch([_preset("ghost_formants", golden_info, irs, full_renders)]))
    torch.cuda.synchronize(0)
    ne = len(eng.last_events(0))
    assert eng.last_grain64(0, ne - 1).size > 0
    for k in (-1, ne):
        with pytest.raises(RuntimeError):
            eng.last_grain64(0, k)
    eng.render_packed(PackedBatch([msgpu.config_params("C2", seed=1000, irs=irs, out_dur_s=0.25)]))
    torch.cuda.synchronize(0)
    with pytest.raises(RuntimeError):
        eng.last_grain64(0, 0)
