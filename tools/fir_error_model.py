#!/usr/bin/env python3
"""Error budget of the space FIR (MS:409-445) in float32, stage by stage.

For a params dict, the oracle's mono (ADSR applied) and the reference's float64
space filter y = IR * (ER cloud) are computed, and y is then recomputed with one
float32 error source at a time (input rounding, tap rounding, float32 FFT
overlap-save with pocketfft's single-precision transforms at the device's block
sizes, filter spectra in float64 vs float32).  Each y goes through the rest of
the output stage (stereo, tanh clip, peak normalise) in float64, and the RMS
distance to the reference's output is printed -- the budget the device's 1e-5
RMS tolerance is spent on.

    python tools/fir_error_model.py ERIR192t2000 ERIR192 ...
"""
import json
import os
import sys

import numpy as np
import scipy.fft as sfft

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "audio-suite_amd"), REPO, os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

from oracle import msound_oracle as O   # noqa: E402


def mono_of(p):
    """The oracle's mono buffer after overlap-add x ADSR (MS:751-764)."""
    plan = O.plan_render(p)
    out = np.zeros(plan.out_n)
    imprint = O.SpectralImprint() if p["spectral_imprint_on"] else None
    prev = None
    for ev in plan.events:
        xg, _ = O.synth_micro(p, ev)
        g = O.spectral_chain(p, ev, xg)
        if p["event_feedback_on"] and prev is not None:
            fb = float(p["event_feedback_amt"])
            L = min(len(g), len(prev))
            g[:L] = (1 - fb) * g[:L] + fb * prev[:L]
        if imprint is not None:
            g = imprint.apply(g, float(p["spectral_imprint_amt"]), float(p["spectral_imprint_smooth"]))
        prev = g.copy()
        if not ev.placed:
            continue
        gg = g[ev.offset:]
        L = min(plan.out_n - ev.start, gg.size)
        if L > 0:
            out[ev.start:ev.start + L] += ev.amp * gg[:L]
    env = O.make_adsr(plan.out_n, plan.base_sr, float(p["env_a"]), float(p["env_d"]), float(p["env_s"]),
                      float(p["env_r"]), float(p["env_curve"]))
    return out * env, plan.base_sr


def space_h(p, n, sr):
    """h = (delta + ER) * IR in float64 (every in-range tap, the whole <= 8192-tap IR)."""
    d = np.zeros(n)
    d[0] = 1.0
    if p["er_cloud_on"]:
        offs, gains = O.er_taps(sr, int(p["er_taps"]), float(p["er_max_ms"]), int(p["seed"]))
        for o, g in zip(offs, gains):
            if 0 < o < n:
                d[o] += g
    ir = O.ir_kernel(p["_ir_audio"][:int(p["space_ir_max_samps"])]) if (p["space_ir_on"] and p.get("_ir_audio") is not None) else None
    last = int(np.nonzero(d)[0].max()) + 1
    h = d[:last] if ir is None else np.convolve(d[:last], ir)
    return h


def tail(p, y, sr):
    st = O.spectral_diffusion_stereo(y, sr, float(p["stereo_width"])) if p["stereo_on"] else np.column_stack([y, y])
    return O.peak_normalize(O.tanh_clip(st, float(p["sat_drive"])), float(p["peak"]))


def ols(x, h, N, P, spec64=False, dtype=np.float32):
    """Overlap-save with Q partitions of P taps, blocks of B = N - P + 1, FFTs in `dtype`."""
    n = x.size
    Q = -(-h.size // P)
    B = N - P + 1
    Hs = []
    for q in range(Q):
        hq = np.zeros(N)
        seg = h[q * P:(q + 1) * P]
        hq[:seg.size] = seg
        Hs.append(np.fft.rfft(hq).astype(np.complex64) if spec64 else sfft.rfft(hq.astype(dtype)))
    xp = np.concatenate([np.zeros(N + Q * P), x.astype(dtype), np.zeros(N)]).astype(dtype)
    base = N + Q * P
    y = np.zeros(n)
    for b in range(-(-n // B)):
        t0 = b * B
        acc = None
        for q in range(Q):
            s = base + t0 - q * P - (P - 1)
            X = sfft.rfft(xp[s:s + N])
            acc = X * Hs[q] if acc is None else acc + X * Hs[q]
        yb = sfft.irfft(acc, n=N)
        m = min(B, n - t0)
        y[t0:t0 + m] = yb[P - 1:P - 1 + m]
    return y


def main(names):
    from conftest import extra_params
    with open(os.path.join(REPO, "tests", "golden", "golden_extra.json")) as fh:
        ge = json.load(fh)
    irs = dict(np.load(os.path.join(REPO, "tests", "golden", "irs.npz")))
    for name in names:
        p = extra_params(ge, irs, name)
        x, sr = mono_of(p)
        n = x.size
        h = space_h(p, n, sr)
        ref_y = np.convolve(x, h)[:n]
        ref = tail(p, ref_y, sr)
        rms = lambda y: float(np.sqrt(np.mean((tail(p, y, sr) - ref) ** 2)))  # noqa: E731
        print(f"{name}: out_n {n}, taps {h.size}, |h|2 {np.linalg.norm(h):.3f}, peak|y| {np.abs(ref_y).max():.3f}")
        print(f"  x -> float32                      {rms(np.convolve(x.astype(np.float32).astype(np.float64), h)[:n]):.3e}")
        print(f"  h -> float32                      {rms(np.convolve(x, h.astype(np.float32).astype(np.float64))[:n]):.3e}")
        print(f"  y -> float32                      {rms(ref_y.astype(np.float32).astype(np.float64)):.3e}")
        for N in (32768, 65536):
            P = (h.size + 1) // 2 if N == 32768 else h.size
            if N == 32768 and P >= N:
                continue
            if N == 65536 and P > 49152:
                continue
            for s64 in (False, True):
                y = ols(x, h, N, min(P, N - 1), spec64=s64)
                print(f"  pocketfft f32 OLS N={N} P={P} H {'f64' if s64 else 'f32'}  {rms(y):.3e}")


if __name__ == "__main__":
    main(sys.argv[1:] or ["ERIR192t2000"])
