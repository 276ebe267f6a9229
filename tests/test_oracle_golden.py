"""Pin the CPU oracle (oracle/msound_oracle.py) to the reference's own outputs.

Golden vectors come from running the reference ``main_v2`` functions in the
survey container (tools/gen_golden.py).  The oracle calls the same NumPy
primitives in the same order, so per-function results must agree to ~1e-12 and
full renders (stored float32) bit-for-bit after the float32 cast.
"""
import hashlib

import numpy as np
import pytest

from oracle import msound_oracle as O
from msgpu.params import config_params, merged

SMALL = [16, 60, 64, 127, 1267, 1500, 2400, 2520]
TOL = 1e-12


def close(a, b, tol=TOL):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    assert np.max(np.abs(a - b), initial=0.0) <= tol * max(1.0, np.max(np.abs(b), initial=0.0))


def test_numpy_stream_pinned(golden_info):
    # Parity is only meaningful on the same PCG64/ziggurat stream.
    got = np.random.default_rng(12345).standard_normal(8).tolist()
    assert got == golden_info["first8_normals_12345"]


@pytest.mark.parametrize("n", SMALL)
def test_spectral_helpers(funcs, n):
    x = funcs[f"in_{n}"]
    close(O.lowpass_fft(x, 1.92e6, 180000.0, roll=25000.0), funcs[f"lowpass_{n}"])
    close(O.lowpass_fft(x, 1.92e6, 180000.0, roll=0.0), funcs[f"lowpass_hard_{n}"])
    close(O.bandpass_fft(x, 960000.0, 40000.0, 160000.0, roll=2000.0), funcs[f"bandpass_{n}"])
    close(O.bandpass_fft(x, 960000.0, 50000.0, 200000.0, roll=0.0), funcs[f"bandpass_hard_{n}"])
    close(O.fft_warp_power(x, 1.25), funcs[f"warp_{n}"])
    for f in (0.5, 0.92, 2.0, 4.0):
        close(O.fft_partial_stretch(x, f), funcs[f"stretch_{f}_{n}"])
    close(O.partial_lock_stretch(x, 1.18, 24, 4), funcs[f"plock_{n}"])
    close(O.cepstral_warp(x, 1.2), funcs[f"cep_{n}"])


@pytest.mark.parametrize("n", SMALL)
def test_models_space_and_feedback(funcs, n):
    x = funcs[f"in_{n}"]
    close(O.resonator_bank(x, 1.2e6, 24, 120, 12000, 80, 77), funcs[f"resbank_{n}"])
    close(O.spectral_diffusion_stereo(x, 48000, 0.65), funcs[f"stereo_{n}"])
    close(O.early_reflection_cloud(x, 48000, 320, 45, 5), funcs[f"er_{n}"])
    close(O.tanh_clip(x, 1.0), funcs[f"softclip_{n}"])
    close(O.peak_normalize(x, 0.98), funcs[f"normalize_{n}"])
    imp = O.SpectralImprint()
    y = np.stack([imp.apply(x, 0.35, 0.92), imp.apply(x[::-1].copy(), 0.35, 0.92)])
    close(y, funcs[f"imprint_{n}"])
    if n >= 64:
        close(O.waveguide_splinters(x, 1.2e6, 8, 1.0, 0.7, 9), funcs[f"waveguide_{n}"])


@pytest.mark.parametrize("n", [12000, 12001])
def test_output_stage_sizes(funcs, irs, n):
    x = funcs[f"in_{n}"]
    close(O.spectral_diffusion_stereo(x, 192000, 0.65), funcs[f"stereo_{n}"])
    close(O.early_reflection_cloud(x, 384000, 320, 45, 1000), funcs[f"er384_{n}"])
    close(O.convolve_ir_short(x, irs["ir_tiny_room_250ms"][:16384]), funcs[f"irconv_{n}"])


@pytest.mark.parametrize("gsr", [48000, 1_920_000, 1_013_600])
def test_generators(funcs, irs, golden_info, gsr):
    for mode in ["Gaussian click", "Dust impulses", "Noise burst", "Skewed transient",
                 "Resonant strike", "bogus"]:
        key = mode.split()[0].lower()
        close(O.gen_basic(gsr, 1.25, 12348, mode, 0.02, -3.0, 4200.0, 12.0),
              funcs[f"gen_{key}_{gsr}"])
    close(O.gen_crackle(gsr, 1.0, 99, 1.4, 180, 64), funcs[f"gen_crackle_{gsr}"])
    close(O.gen_stick_slip(gsr, 1.2, 99, 0.9, 0.06, 0.75, 0.08), funcs[f"gen_stickslip_{gsr}"])
    close(O.gen_micro_chaos(gsr, 0.9, 99, 3.92, 0.35), funcs[f"gen_chaos_{gsr}"])
    key = f"gen_wavelet_{gsr}"
    if key in golden_info["func_errors"]:
        with pytest.raises(ValueError):
            O.gen_wavelet_atoms(gsr, 1.5, 99, 2400.0, 8, 0.6)
    else:
        close(O.gen_wavelet_atoms(gsr, 1.5, 99, 2400.0, 8, 0.6), funcs[key])
    close(O.gen_ir_fragment(irs["tiny_room_ir"], gsr, 2.0, 99)[0], funcs[f"gen_irfrag_{gsr}"])


def test_adsr_events_breakpoints(funcs):
    for i in range(5):
        n, sr, a, d, s, r, c = funcs[f"adsr_args_{i}"]
        close(O.make_adsr(int(n), sr, a, d, s, r, c), funcs[f"adsr_{i}"])
    for proc in ("Single", "Poisson", "Clustered", "Hawkes"):
        for seed in (12345, 1000, 77):
            t = O.generate_event_times(proc, 8.0, 18.0, seed, 6, 25.0, 0.6, 0.25)
            close(np.asarray(t, dtype=np.float64), funcs[f"events_{proc}_{seed}"], 0.0)
    pts = O.parse_breakpoints("0:18, 4:40, 8:14")
    got = [O.eval_breakpoints(pts, t, 3.0) for t in funcs["bp_t"]]
    close(got, funcs["bp_eval"], 0.0)
    with pytest.raises(ValueError):
        O.parse_breakpoints("1:2:3")


def _render_f32(p):
    audio, meta = O.render(p)
    return audio.astype(np.float32), meta


@pytest.mark.parametrize("name,cfg,kw", [
    ("C1", "C1", {}), ("C2", "C2", {}), ("C3", "C3", {}),
    ("C3s1001", "C3", dict(seed=1001, out_dur_s=0.25)),
    ("C4s1000short", "C4", dict(out_dur_s=0.25)),
    ("C2odd", "C2", dict(seed=1002, out_dur_s=0.5 + 1 / 192000)),
])
def test_full_render_configs(full_renders, irs, name, cfg, kw):
    kw = dict(kw)
    seed = kw.pop("seed", 1000)
    p = config_params(cfg, seed=seed, irs=irs, **kw)
    a, meta = _render_f32(p)
    close(a, full_renders[f"{name}_audio"], 2e-7)
    assert meta["design_sr_base"] == int(full_renders[f"{name}_design_sr"])
    for k in ("micro_last", "grain_last"):
        key = f"{name}_{k}"
        if key in full_renders.files:
            close(meta[k], full_renders[key])


def test_defaults_render(full_renders):
    p = dict(merged(out_dur_s=0.5), _ir_audio=None, _img_gray=None)
    a, _ = _render_f32(p)
    close(a, full_renders["defaults_short_audio"], 2e-7)


def test_presets_render(full_renders, irs, golden_info):
    img = full_renders["image_gray"]
    for name in golden_info["presets"]:
        p = merged(golden_info["preset_params"][name])
        p["out_dur_s"] = 0.5
        p["_ir_audio"] = irs["tiny_room_ir"]
        p["_img_gray"] = img
        a, _ = _render_f32(p)
        close(a, full_renders[f"preset_{name}_audio"], 2e-7)


def test_c3_summaries(irs, golden_info):
    for seed in (1000, 1001):
        a, _ = O.render(config_params("C3", seed=seed, irs=irs))
        s = golden_info["summaries"][f"C3_{seed}"]
        assert hashlib.sha1(a.astype(np.float32).tobytes()).hexdigest() == s["sha1_f32"]


def test_c4_c5_decimated(irs, large_renders, golden_info):
    for name in ("C4", "C5"):
        a, _ = O.render(config_params(name, seed=1000, irs=irs))
        step = int(large_renders[f"{name}_step"])
        close(a[::step].astype(np.float32), large_renders[f"{name}_dec"], 2e-7)
        close(a[:8192].astype(np.float32), large_renders[f"{name}_head"], 2e-7)
        close(a[-8192:].astype(np.float32), large_renders[f"{name}_tail"], 2e-7)
        s = golden_info["summaries"][f"{name}_1000"]
        assert abs(float(np.sqrt(np.mean(a ** 2))) - s["rms"]) < 1e-12


def test_stft_mag_db_pinned():
    """The oracle's spectrogram helper against the reference's (MS:197-212)."""
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "stft.npz"))
    for name in ("c2", "defaults", "capped", "short", "odd"):
        sr, win, hop, mf = (int(v) for v in z[f"{name}_cfg"])
        S = O.stft_mag_db(z[f"{name}_x"], sr, win=win, hop=hop, max_frames=mf)
        assert S.shape == z[f"{name}_S"].shape
        assert np.max(np.abs(S.astype(np.float32) - z[f"{name}_S"])) <= 1e-3, name


def test_fir_causal_is_the_capped_ir_convolution():
    """fir_causal is convolve_ir_short's arithmetic (MS:438-445) for IRs inside the 8192 cap."""
    rng = np.random.default_rng(5)
    x = rng.standard_normal(3000)
    ir = O.peak_normalize(rng.standard_normal(700), 0.9)
    np.testing.assert_array_equal(O.fir_causal(x, O.ir_kernel(ir)), O.convolve_ir_short(x, ir))
    h = O.synthetic_fir_taps(16384)
    assert h.shape == (16384,) and abs(np.max(np.abs(h)) - 0.9) < 1e-12


@pytest.mark.parametrize("name", ["ERIR192", "ERIR192t2000", "ERIR176", "ER384", "H48_1000"])
def test_extra_renders(irs, extra_renders, golden_extra, name):
    """Round-3 goldens (tools/gen_golden_r3.py): space filters longer than one
    32 768-point transform and the H48 metric point, whole buffers."""
    from conftest import extra_params
    a, _ = _render_f32(extra_params(golden_extra, irs, name))
    close(a, extra_renders[f"{name}_audio"], 2e-7)


def test_extra_h48_summaries(irs, golden_extra):
    from conftest import extra_params
    for s in (1001, 1002, 1003):
        a, _ = O.render(extra_params(golden_extra, irs, f"H48_{s}"))
        g = golden_extra["summaries"][f"H48_{s}"]
        assert hashlib.sha1(a.astype(np.float32).tobytes()).hexdigest() == g["sha1_f32"]


@pytest.mark.slow
def test_extra_odd_stereo_long(irs, extra_renders, golden_extra):
    """ODD44: the oracle's odd-length rotation at 4 200 525 frames."""
    from conftest import extra_params
    a, _ = O.render(extra_params(golden_extra, irs, "ODD44"))
    step = int(golden_extra["decimation"])
    close(a[::step].astype(np.float32), extra_renders["ODD44_dec"], 2e-7)
    close(a[-8192:].astype(np.float32), extra_renders["ODD44_tail"], 2e-7)


def _progress_params(case, irs, img):
    p = merged(case["params"])
    p["_img_gray"] = img if case["image"] else None
    p["_ir_audio"] = irs["tiny_room_ir"] if case["ir"] else None
    return p


def test_progress_messages_pinned(irs, full_renders):
    """The oracle's progress messages equal the reference's (tests/golden/progress.json):
    the SR line, every 50th event with its generator note (Image line y=..., IR
    fragment, no-source notes, MS:342-362, 757-758) and Done."""
    import json
    import os
    cases = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "progress.json")))
    for name, case in cases.items():
        msgs = []
        O.render(_progress_params(case, irs, full_renders["image_gray"]),
                 progress=lambda v, m: msgs.append([int(v), str(m)]))
        assert msgs == case["messages"], name


def test_long_fixture_is_the_references():
    """the > 2^29-frame fixture is the reference's own render
    (tools/gen_golden_r5.py imports main_v2.render), and the NumPy restatement's
    summary of the same dict was equal to it in every field."""
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "long_2e29.json")) as f:
        g = json.load(f)
    assert g["source"].startswith("reference: microsound_0.2.1/main_v2.py")
    assert g["out_n"] == (1 << 29) + (1 << 18)
    assert g["oracle_equal"] and all(g["oracle_equal"].values())
