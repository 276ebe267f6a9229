#!/usr/bin/env python3
"""Generate golden vectors by importing the reference Microsound ``render``.

Container-only tool (``/root/reference`` does not exist on the GPU box).  It
imports ``microsound_0.2.1/main_v2.py`` with the three GUI/IO modules it never
uses on the render path (PyQt6, pyqtgraph, soundfile) stubbed, calls the
reference's own functions, and writes DATA fixtures (inputs + expected outputs)
under ``tests/golden/``.  No reference source is copied.

    python tools/gen_golden.py            # all fixtures (C5 takes ~30 s)
    python tools/gen_golden.py --quick    # skip C4/C5 summaries
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import sys
import time
import types

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference

import numpy as np
from scipy.io import wavfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_DIR = "/root/reference/microsound_0.2.1"
OUT = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))

from msgpu.params import DEFAULTS, CONFIGS, config_params, merged  # noqa: E402


def import_reference():
    def stub(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class QObject:  # RenderWorker base; never instantiated here
        pass

    qc = stub("PyQt6.QtCore", QObject=QObject, pyqtSignal=lambda *a, **k: None,
              pyqtSlot=lambda *a, **k: (lambda f: f))
    qw = stub("PyQt6.QtWidgets", QMainWindow=object)
    stub("PyQt6", QtCore=qc, QtWidgets=qw)
    stub("pyqtgraph")
    stub("soundfile")
    sys.path.insert(0, REF_DIR)
    import main_v2  # noqa: E402
    return main_v2


def load_irs():
    """IRs as the UI loads them (MS:1405-1409): PCM16/32768 -> mono -> normalize(0.9)."""
    irs = {}
    for f in sorted(glob.glob(os.path.join(REF_DIR, "irs", "*.wav"))):
        sr, a = wavfile.read(f)
        assert a.dtype == np.int16 and sr == 48000
        x = a.astype(np.float64) / 32768.0
        if x.ndim > 1:
            x = x.mean(axis=1)
        m = float(np.max(np.abs(x)))
        x = x * (0.9 / m)
        irs[os.path.splitext(os.path.basename(f))[0]] = x
    return irs


def summary(a: np.ndarray) -> dict:
    a32 = np.ascontiguousarray(a, dtype=np.float32)
    return {
        "shape": list(a.shape),
        "sha1_f32": hashlib.sha1(a32.tobytes()).hexdigest(),
        "rms": float(np.sqrt(np.mean(a.astype(np.float64) ** 2))),
        "peak": float(np.max(np.abs(a))),
        "sum_l": float(np.sum(a[:, 0], dtype=np.float64)),
        "sum_r": float(np.sum(a[:, 1], dtype=np.float64)),
    }


class _Errors(dict):
    pass


ERRORS = _Errors()


def func_cases(ms, irs):
    """Per-function goldens at small and awkward sizes.

    A reference call that raises is recorded in ERRORS (name -> exception type),
    so the restatement can be checked to raise the same way.
    """
    class Out(dict):
        def set(self, key, fn, *a, **k):
            try:
                self[key] = fn(*a, **k)
            except Exception as e:  # reference behaviour to reproduce
                ERRORS[key] = type(e).__name__
    out = Out()
    sizes = [16, 60, 64, 127, 1267, 1500, 2400, 2520]
    for n in sizes:
        rng = np.random.default_rng(1000 + n)
        x = rng.standard_normal(n)
        out[f"in_{n}"] = x
        out[f"lowpass_{n}"] = ms.lowpass_fft(x, 1.92e6, 18000.0 * 10, roll=2500.0 * 10)
        out[f"lowpass_hard_{n}"] = ms.lowpass_fft(x, 1.92e6, 180000.0, roll=0.0)
        out[f"bandpass_{n}"] = ms.bandpass_fft(x, 960000.0, 2000.0 * 20, 8000.0 * 20, roll=2000.0)
        out[f"bandpass_hard_{n}"] = ms.bandpass_fft(x, 960000.0, 50000.0, 200000.0, roll=0.0)
        out[f"warp_{n}"] = ms.fft_warp_power(x, 1.25)
        for f in (0.5, 0.92, 2.0, 4.0):
            out[f"stretch_{f}_{n}"] = ms.fft_partial_stretch(x, f)
        out[f"plock_{n}"] = ms.partial_lock_stretch(x, 1.18, top_n=24, neighborhood=4)
        out[f"cep_{n}"] = ms.cepstral_warp(x, 1.2)
        out[f"resbank_{n}"] = ms.resonator_bank(x, 1.2e6, modes=24, f_min=120, f_max=12000,
                                                decay_ms=80, seed=77)
        out[f"stereo_{n}"] = ms.spectral_diffusion_stereo(x, 48000, width=0.65)
        out[f"er_{n}"] = ms.early_reflection_cloud(x, 48000, taps=320, max_ms=45, seed=5)
        out[f"softclip_{n}"] = ms.soft_clip(x, 1.0)
        out[f"normalize_{n}"] = ms.normalize(x, 0.98)
        imp = ms.SpectralImprint()
        y1 = imp.apply(x, 0.35, 0.92)
        y2 = imp.apply(x[::-1].copy(), 0.35, 0.92)
        out[f"imprint_{n}"] = np.stack([y1, y2])
        if n >= 64:
            out[f"waveguide_{n}"] = ms.waveguide_splinters(x, 1.2e6, lines=8, max_ms=1.0,
                                                           feedback=0.7, seed=9)
    # long stereo / FIR cases at output-stage sizes, even and odd
    for n in (12000, 12001):
        x = np.random.default_rng(n).standard_normal(n)
        out[f"in_{n}"] = x
        out[f"stereo_{n}"] = ms.spectral_diffusion_stereo(x, 192000, width=0.65)
        out[f"er384_{n}"] = ms.early_reflection_cloud(x, 384000, taps=320, max_ms=45, seed=1000)
        out[f"irconv_{n}"] = ms.convolve_ir_short(x, irs["ir_tiny_room_250ms"][:16384])
    # generators: every mode, design SRs giving awkward n
    gen_modes = ["Gaussian click", "Dust impulses", "Noise burst", "Skewed transient",
                 "Resonant strike", "bogus"]
    for gsr in (48000, 1_920_000, 1_013_600):
        for mode in gen_modes:
            key = mode.split()[0].lower()
            out[f"gen_{key}_{gsr}"] = ms.gen_basic(gsr, 1.25, 12345 + 3, mode, 0.02, -3.0, 4200.0, 12.0)
        out[f"gen_crackle_{gsr}"] = ms.gen_crackle(gsr, 1.0, 99, alpha=1.4, density=180, kernel=64)
        out[f"gen_stickslip_{gsr}"] = ms.gen_stick_slip(gsr, 1.2, 99, 0.9, 0.06, 0.75, 0.08)
        out[f"gen_chaos_{gsr}"] = ms.gen_micro_chaos(gsr, 0.9, 99, r=3.92, gate=0.35)
        out.set(f"gen_wavelet_{gsr}", ms.gen_wavelet_atoms, gsr, 1.5, 99, 2400.0, 8, 0.6)
        out[f"gen_irfrag_{gsr}"] = ms.gen_ir_fragment(irs["tiny_room_ir"], gsr, 2.0, 99)[0]
    # ADSR: several shapes incl. release > n, zero stages
    for i, (n, sr, a, d, s, r, c) in enumerate([
            (48000, 48000, 20, 250, 0.65, 1800, 1.8), (384000, 384000, 20, 250, 0.65, 1800, 1.8),
            (1000, 48000, 0, 0, 0.5, 0, 1.0), (96000, 48000, 100, 300, 0.2, 500, 3.0),
            (5000, 48000, 10, 2000, 1.0, 10, 0.5)]):
        out[f"adsr_{i}"] = ms.make_adsr(n, sr, a, d, s, r, c)
        out[f"adsr_args_{i}"] = np.array([n, sr, a, d, s, r, c], dtype=np.float64)
    # event fields
    for proc in ("Single", "Poisson", "Clustered", "Hawkes"):
        for seed in (12345, 1000, 77):
            t = ms.generate_event_times(proc, 8.0, 18.0, seed, 6, 25.0, 0.6, 0.25)
            out[f"events_{proc}_{seed}"] = np.asarray(t, dtype=np.float64)
    # breakpoints
    pts = ms.parse_breakpoints("0:18, 4:40, 8:14")
    ts = np.linspace(-1, 10, 45)
    out["bp_eval"] = np.array([ms.eval_breakpoints(pts, t, 3.0) for t in ts])
    out["bp_t"] = ts
    return out


def render_case(ms, p):
    t0 = time.time()
    audio, meta = ms.render(p)
    dt = time.time() - t0
    return audio, meta, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    args = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    ms = import_reference()
    irs = load_irs()
    np.savez_compressed(os.path.join(OUT, "irs.npz"), **irs)

    info = {"numpy": np.__version__,
            "first8_normals_12345": np.random.default_rng(12345).standard_normal(8).tolist(),
            "reference": "microsound_0.2.1/main_v2.py",
            "generator": "tools/gen_golden.py"}

    fc = func_cases(ms, irs)
    np.savez_compressed(os.path.join(OUT, "funcs.npz"), **fc)
    print(f"funcs.npz: {len(fc)} arrays")

    # Full-buffer renders (stored float32) -----------------------------------
    full = {}
    timings = {}
    cases = {
        "C1": config_params("C1", seed=1000, irs=irs),
        "C2": config_params("C2", seed=1000, irs=irs),
        "C3": config_params("C3", seed=1000, irs=irs),
        "C3s1001": config_params("C3", seed=1001, irs=irs, out_dur_s=0.25),
        "C4s1000short": config_params("C4", seed=1000, irs=irs, out_dur_s=0.25),
        "defaults_short": dict(merged(out_dur_s=0.5), _ir_audio=None, _img_gray=None),
        "C2odd": config_params("C2", seed=1002, irs=irs, out_dur_s=0.5 + 1 / 192000),
    }
    for name, p in cases.items():
        audio, meta, dt = render_case(ms, p)
        full[f"{name}_audio"] = audio.astype(np.float32)
        for k in ("micro_last", "grain_last"):
            if meta.get(k) is not None:
                full[f"{name}_{k}"] = np.asarray(meta[k], dtype=np.float64)
        full[f"{name}_design_sr"] = np.array(meta["design_sr_base"])
        timings[name] = dt
        print(f"{name}: {audio.shape} {dt:.2f}s")

    # Presets merged over factory defaults, shortened to 0.5 s -----------------
    img = (np.add.outer(np.arange(48), np.arange(64)) * 7 % 256).astype(np.uint8)
    full["image_gray"] = img
    preset_names = []
    for f in sorted(glob.glob(os.path.join(REF_DIR, "presets", "*.json"))):
        name = os.path.splitext(os.path.basename(f))[0]
        with open(f, "r", encoding="utf-8") as fh:
            pr = json.load(fh)
        p = merged(pr)
        p["out_dur_s"] = 0.5
        p["_ir_audio"] = irs["tiny_room_ir"]
        p["_img_gray"] = img
        audio, meta, dt = render_case(ms, p)
        full[f"preset_{name}_audio"] = audio.astype(np.float32)
        preset_names.append(name)
        timings[f"preset_{name}"] = dt
        print(f"preset {name}: {audio.shape} {dt:.2f}s")
    np.savez_compressed(os.path.join(OUT, "render_full.npz"), **full)
    info["presets"] = preset_names
    info["preset_params"] = {}
    for f in sorted(glob.glob(os.path.join(REF_DIR, "presets", "*.json"))):
        with open(f, "r", encoding="utf-8") as fh:
            info["preset_params"][os.path.splitext(os.path.basename(f))[0]] = json.load(fh)

    # Summaries at BASELINE sizes ----------------------------------------------
    summ = {}
    dec = {}
    seeds = [1000, 1001, 1002, 1003]
    for s in seeds:
        p = config_params("C3", seed=s, irs=irs)
        audio, meta, dt = render_case(ms, p)
        summ[f"C3_{s}"] = summary(audio)
        timings[f"C3_{s}"] = dt
    if not args.quick:
        for name, dstep in (("C4", 16), ("C5", 256)):
            p = config_params(name, seed=1000, irs=irs)
            audio, meta, dt = render_case(ms, p)
            summ[f"{name}_1000"] = summary(audio)
            dec[f"{name}_dec"] = audio[::dstep].astype(np.float32)
            dec[f"{name}_head"] = audio[:8192].astype(np.float32)
            dec[f"{name}_tail"] = audio[-8192:].astype(np.float32)
            dec[f"{name}_step"] = np.array(dstep)
            timings[f"{name}_1000"] = dt
            print(f"{name}: {audio.shape} {dt:.2f}s")
        np.savez_compressed(os.path.join(OUT, "render_large.npz"), **dec)
    info["summaries"] = summ
    info["func_errors"] = dict(ERRORS)
    info["timings_s"] = timings
    with open(os.path.join(OUT, "golden_info.json"), "w") as fh:
        json.dump(info, fh, indent=1, ensure_ascii=False)
    print("done")


if __name__ == "__main__":
    main()
