"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

A NumPy restatement of the Microsound render path of the reference
(``microsound_0.2.1/main_v2.py``, cited as ``MS:<line>``), organised the way the
MI355X build executes it: a *plan* (all scalar/RNG decisions per event and per
render), a per-event *grain* stage, and the *output* stage.  It is used only by
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of
``bench.py`` as the checker / CPU baseline — never by the product path
(``msgpu``), which fails loudly when the HIP library is missing.

Pinning: every function is checked against golden vectors produced by the
reference itself (``tools/gen_golden.py`` imports ``main_v2`` with GUI stubs) in
``tests/test_oracle_golden.py``; tolerance 1e-12 (same float64 NumPy ops).

Third-party arithmetic: NumPy 2.2.6 (pocketfft ``rfft/irfft``, ``convolve``,
``interp`` and the ``Generator``/PCG64 streams) — the same library the reference
calls, so the restatement calls it too.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

GEN_SR_CAP = 30_000_000  # MS:597 / MS:646
IR_TAP_CAP = 8192        # MS:443

BASIC_MODES = ("Gaussian click", "Dust impulses", "Noise burst", "Skewed transient",
               "Resonant strike")  # MS:652


# ---------------------------------------------------------------------------
# L1 elementwise helpers
# ---------------------------------------------------------------------------
def hann(n: int) -> np.ndarray:
    """Symmetric Hann window (MS:17-21)."""
    if n <= 1:
        return np.ones(n, dtype=np.float64)
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2 * np.pi * k / (n - 1))


def peak_normalize(x: np.ndarray, peak: float = 0.98) -> np.ndarray:
    """Scale so max|x| == peak; all-zero input returned as is (MS:26-29)."""
    m = float(np.max(np.abs(x))) if x.size else 0.0
    return x if m <= 0 else x * (peak / m)


def tanh_clip(x: np.ndarray, drive: float = 1.0) -> np.ndarray:
    """tanh(x*d)/tanh(d) for d > 0, identity otherwise (MS:31-34)."""
    d = float(drive)
    return x if d <= 0 else np.tanh(x * d) / np.tanh(d)


def bin_freqs(n: int, sr: float) -> np.ndarray:
    """rFFT bin centre frequencies, ``rfftfreq(n, 1/sr)`` (MS:36-37)."""
    return np.fft.rfftfreq(n, d=1.0 / sr)


def _interp_complex(k_in: np.ndarray, k: np.ndarray, X: np.ndarray) -> np.ndarray:
    """Linear interpolation of re and im separately, zero outside (MS:112-114, 125-127)."""
    re = np.interp(k_in, k, X.real, left=0.0, right=0.0)
    im = np.interp(k_in, k, X.imag, left=0.0, right=0.0)
    return re + 1j * im


# ---------------------------------------------------------------------------
# Spectral masks (MS:39-101) — written as real per-bin weights
# ---------------------------------------------------------------------------
def lowpass_fft(x: np.ndarray, sr: float, cutoff: float, roll: float = 0.0) -> np.ndarray:
    """Brick-wall / cosine-roll FFT low-pass (MS:39-59)."""
    n = len(x)
    if n < 8:
        return x
    nyq = 0.5 * sr
    c = float(np.clip(cutoff, 1.0, nyq))
    r = float(max(0.0, roll))
    X = np.fft.rfft(x)
    f = bin_freqs(n, sr)
    if r <= 0:
        X[f > c] = 0.0
    else:
        f1 = min(nyq, c + r)
        X[f > f1] = 0.0
        band = (f >= c) & (f <= f1)
        if np.any(band):
            t = (f[band] - c) / max(1e-12, (f1 - c))
            X[band] *= 0.5 * (1.0 + np.cos(np.pi * t))   # 1 -> 0 across [c, f1]
    return np.fft.irfft(X, n=n).astype(np.float64, copy=False)


def bandpass_fft(x: np.ndarray, sr: float, lo: float, hi: float, roll: float = 0.0) -> np.ndarray:
    """Raised-cosine FFT band-pass used by the multi-band unfold (MS:61-101)."""
    n = len(x)
    if n < 8:
        return x
    lo = max(0.0, float(lo))
    hi = max(lo, float(hi))
    X = np.fft.rfft(x)
    f = bin_freqs(n, sr)
    nyq = 0.5 * sr
    hi = min(hi, nyq)
    if hi <= 0:
        return np.zeros_like(x)
    r = float(max(0.0, roll))
    Y = X.copy()
    if lo > 0:                                    # rising edge below lo (MS:74-86)
        if r <= 0:
            Y[f < lo] = 0.0
        else:
            f0, f1 = max(0.0, lo - r), lo
            Y[f < f0] = 0.0
            band = (f >= f0) & (f <= f1)
            if np.any(band):
                t = (f[band] - f0) / max(1e-12, (f1 - f0))
                Y[band] *= 0.5 * (1.0 - np.cos(np.pi * t))
    if hi < nyq:                                  # falling edge above hi (MS:88-100)
        if r <= 0:
            Y[f > hi] = 0.0
        else:
            f0, f1 = hi, min(nyq, hi + r)
            Y[f > f1] = 0.0
            band = (f >= f0) & (f <= f1)
            if np.any(band):
                t = (f[band] - f0) / max(1e-12, (f1 - f0))
                Y[band] *= 0.5 * (1.0 + np.cos(np.pi * t))
    return np.fft.irfft(Y, n=n).astype(np.float64, copy=False)


# ---------------------------------------------------------------------------
# Spectral warps (MS:103-163)
# ---------------------------------------------------------------------------
def fft_warp_power(x: np.ndarray, power: float) -> np.ndarray:
    """Bin remap k_in = (k/kmax)^(1/p) * kmax (MS:103-115)."""
    n = len(x)
    if n < 16:
        return x
    X = np.fft.rfft(x)
    k = np.arange(X.size, dtype=np.float64)
    kmax = max(1.0, k[-1])
    k_in = np.power(k / kmax, 1.0 / max(1e-6, float(power))) * kmax
    return np.fft.irfft(_interp_complex(k_in, k, X), n=n).astype(np.float64, copy=False)


def fft_partial_stretch(x: np.ndarray, factor: float) -> np.ndarray:
    """Spectral stretch Y[k] = X(k/factor) (MS:117-128)."""
    n = len(x)
    if n < 16:
        return x
    factor = float(factor)
    if abs(factor - 1.0) < 1e-9:
        return x
    X = np.fft.rfft(x)
    k = np.arange(X.size, dtype=np.float64)
    Y = _interp_complex(k / max(1e-12, factor), k, X)
    return np.fft.irfft(Y, n=n).astype(np.float64, copy=False)


def partial_lock_stretch(x: np.ndarray, factor: float, top_n: int = 24,
                         neighborhood: int = 4) -> np.ndarray:
    """Move the top-N magnitude bins to round(k*factor) with a triangular spread (MS:130-148)."""
    n = len(x)
    if n < 64:
        return x
    factor = float(factor)
    if abs(factor - 1.0) < 1e-9:
        return x
    X = np.fft.rfft(x)
    K = X.size
    peaks = np.argsort(np.abs(X)[1:])[-top_n:] + 1
    Y = np.zeros_like(X)
    for k in peaks:                       # accumulation order = argsort order
        k2 = int(round(k * factor))
        if not (1 <= k2 < K):
            continue
        for d in range(-neighborhood, neighborhood + 1):
            kk = k2 + d
            if 1 <= kk < K:
                Y[kk] += X[k] * (1.0 - (abs(d) / (neighborhood + 1)))
    Y += 0.12 * X
    return np.fft.irfft(Y, n=n).astype(np.float64)


def cepstral_warp(x: np.ndarray, factor: float) -> np.ndarray:
    """Warp the real cepstrum by t/factor, keep the phase (MS:150-163)."""
    n = len(x)
    if n < 64:
        return x
    X = np.fft.rfft(x)
    cep = np.fft.irfft(np.log(np.abs(X) + 1e-12), n=n)
    t = np.arange(n, dtype=np.float64)
    cep2 = np.interp(t / max(1e-12, float(factor)), t, cep, left=0.0, right=0.0)
    mag2 = np.exp(np.fft.rfft(cep2).real)
    return np.fft.irfft(mag2 * np.exp(1j * np.angle(X)), n=n).astype(np.float64)


# ---------------------------------------------------------------------------
# Envelope (MS:172-195)
# ---------------------------------------------------------------------------
def make_adsr(n, sr, A_ms, D_ms, S, R_ms, curve=1.8):
    """Piecewise ADSR with power-curve segments (MS:172-195)."""
    A = max(0, int(round(sr * A_ms / 1000.0)))
    D = max(0, int(round(sr * D_ms / 1000.0)))
    R = max(0, int(round(sr * R_ms / 1000.0)))
    S = float(np.clip(S, 0, 1))
    c = float(max(1e-6, curve))
    env = np.ones(n, dtype=np.float64)
    i = 0
    if A > 0:
        env[:A] = np.linspace(0, 1, A, endpoint=False) ** c   # raises if A > n (MS:182)
        i = A
    j = min(n, i + D)
    if D > 0 and j > i:
        env[i:j] = 1.0 - (1.0 - S) * (np.linspace(0, 1, j - i, endpoint=False) ** c)
    s0, s1 = j, max(j, n - R)
    if s1 > s0:
        env[s0:s1] = S
    if R > 0 and n > s1:
        env[s1:] = S * (1.0 - (np.linspace(0, 1, n - s1, endpoint=True) ** c))
    return env


def morlet_atom(gen_sr, dur_ms, f0, sigma_ms, phase=0.0):
    """Gaussian-windowed cosine centred at n/2 (MS:165-170)."""
    n = int(max(16, round(gen_sr * dur_ms / 1000.0)))
    t = (np.arange(n, dtype=np.float64) - (n / 2)) / gen_sr
    s = max(1e-9, (sigma_ms / 1000.0))
    return (np.exp(-0.5 * (t / s) ** 2) * np.cos(2 * np.pi * f0 * t + phase)).astype(np.float64)


# ---------------------------------------------------------------------------
# Generators (MS:219-362)
# ---------------------------------------------------------------------------
def grain_len(gen_sr: int, micro_ms: float, floor: int = 16) -> int:
    """Samples per micro event at design SR (MS:221, 273, 285, 305, 319, 337, 352)."""
    return int(max(floor, round(gen_sr * micro_ms / 1000.0)))


def gen_basic(gen_sr, micro_ms, seed, mode, dust_density, noise_tilt_db_oct,
              ring_hz, ring_decay_ms):
    """The five closed-form modes + noise fallback, then edge fades (MS:219-269)."""
    rng = np.random.default_rng(int(seed))
    n = grain_len(gen_sr, micro_ms)
    t = np.arange(n, dtype=np.float64) / gen_sr

    def tilted(nn, tilt):                          # MS:224-233
        w = rng.standard_normal(nn).astype(np.float64)
        W = np.fft.rfft(w)
        f = bin_freqs(nn, gen_sr)
        if f.size > 1:
            f[0] = f[1]
        alpha = math.log(10.0 ** (tilt / 20.0), 2.0)
        W *= (f / max(1e-12, f[1])) ** alpha
        return np.fft.irfft(W, n=nn).astype(np.float64)

    if mode == "Gaussian click":
        sigma = max(1, int(0.0025 * n))
        x = np.exp(-0.5 * ((np.arange(n) / sigma) ** 2)) * (rng.standard_normal(n) * 0.12 + 1.0)
    elif mode == "Dust impulses":
        x = np.zeros(n, dtype=np.float64)
        k = int(max(1, round(dust_density * n)))
        idx = rng.integers(0, n, size=k)
        x[idx] = rng.uniform(-1, 1, size=k)
        x = np.convolve(x, np.exp(-np.linspace(0, 6, max(8, int(0.01 * n)))), mode="same")
    elif mode == "Noise burst":
        x = tilted(n, noise_tilt_db_oct) * np.exp(-t / max(1e-6, (micro_ms / 1000.0) * 0.25))
    elif mode == "Skewed transient":
        w = np.maximum(0.0, tilted(n, noise_tilt_db_oct))
        x = np.diff(w, prepend=w[0]) * np.exp(-t / max(1e-6, (micro_ms / 1000.0) * 0.2))
    elif mode == "Resonant strike":
        f = max(10.0, float(ring_hz))
        tau = max(1e-6, float(ring_decay_ms) / 1000.0)
        ring = np.sin(2 * np.pi * f * t) * np.exp(-t / tau)
        exc = rng.standard_normal(n) * np.exp(-t / max(1e-6, (micro_ms / 1000.0) * 0.15))
        x = 0.9 * ring + 0.25 * exc
    else:
        x = rng.standard_normal(n).astype(np.float64) * 0.1
    return (x * edge_fade(n)).astype(np.float64)


def edge_fade(n: int) -> np.ndarray:
    """Linear fade-in/out of max(8, int(0.01 n)) samples (MS:265-268)."""
    fade = max(8, int(0.01 * n))
    w = np.ones(n, dtype=np.float64)
    w[:fade] *= np.linspace(0, 1, fade, endpoint=False)
    w[-fade:] *= np.linspace(1, 0, fade, endpoint=False)
    return w


def gen_crackle(gen_sr, micro_ms, seed, alpha=1.4, density=180, kernel=64):
    """Pareto-spaced impulses convolved with an exp kernel (MS:271-281)."""
    rng = np.random.default_rng(int(seed))
    n = grain_len(gen_sr, micro_ms)
    x = np.zeros(n, dtype=np.float64)
    times = np.cumsum(rng.pareto(alpha, int(max(8, density))))
    for ti in times[times < n].astype(int):
        x[ti] += rng.uniform(-1, 1)
    return np.convolve(x, np.exp(-np.linspace(0, 6, max(8, int(kernel)))), mode="same").astype(np.float64)


def gen_stick_slip(gen_sr, micro_ms, seed, threshold=0.9, build=0.06, decay=0.75, noise=0.08):
    """Stick/slip force state machine, Hann-windowed (MS:283-301)."""
    rng = np.random.default_rng(int(seed))
    n = grain_len(gen_sr, micro_ms, 64)
    x = np.zeros(n, dtype=np.float64)
    stuck, force = True, 0.0
    for i in range(n):
        if stuck:
            force += build * (rng.standard_normal() * noise + 0.2)
            if abs(force) > threshold:
                stuck = False
        else:
            x[i] = force + 0.25 * rng.standard_normal()
            force *= decay
            if abs(force) < 0.02:
                stuck, force = True, 0.0
    x *= hann(n)
    return x.astype(np.float64)


def gen_micro_chaos(gen_sr, micro_ms, seed, r=3.92, gate=0.35):
    """Gated logistic map, exp-smoothed and Hann-windowed (MS:303-315)."""
    rng = np.random.default_rng(int(seed))
    n = grain_len(gen_sr, micro_ms, 64)
    x = np.zeros(n, dtype=np.float64)
    y = (int(seed) % 10000) / 10000.0
    for i in range(n):
        y = r * y * (1.0 - y)
        if rng.random() < gate:
            x[i] = y - 0.5
    x = np.convolve(x, np.exp(-np.linspace(0, 5, 48)), mode="same")
    x *= hann(n)
    return x.astype(np.float64)


def gen_wavelet_atoms(gen_sr, micro_ms, seed, base_hz=2400, count=8, spread=0.6):
    """Sum of randomly shifted Morlet atoms, Hann-windowed (MS:317-331)."""
    rng = np.random.default_rng(int(seed))
    n = grain_len(gen_sr, micro_ms, 128)
    x = np.zeros(n, dtype=np.float64)
    for k in range(int(max(1, count))):
        f0 = base_hz * (2.0 ** rng.uniform(-spread, spread))
        sigma_ms = max(0.03, micro_ms * rng.uniform(0.04, 0.18))
        phase = rng.uniform(0, 2 * np.pi)
        atom = morlet_atom(gen_sr, dur_ms=micro_ms, f0=f0, sigma_ms=sigma_ms, phase=phase)
        atom = np.roll(atom, int(rng.integers(-n // 8, n // 8)))
        x += (1.0 / (1 + k * 0.6)) * atom[:n]   # ValueError when the atom is shorter (MS:329)
    x *= hann(n)
    return x.astype(np.float64)


def gen_ir_fragment(ir_audio, gen_sr, micro_ms, seed):
    """A random 256-sample IR slice stretched to n, Hann, normalised to 0.9 (MS:333-348)."""
    rng = np.random.default_rng(int(seed))
    if ir_audio is None or ir_audio.size < 32:
        return np.zeros(grain_len(gen_sr, micro_ms)), "No IR loaded"
    n = grain_len(gen_sr, micro_ms, 64)
    src = ir_audio.astype(np.float64)
    if src.ndim > 1:
        src = src.mean(axis=1)
    start = rng.integers(0, max(1, src.size - 256))
    sl = src[start:start + 256]
    x = np.interp(np.linspace(0, 1, n), np.linspace(0, 1, sl.size), sl)
    x *= hann(n)
    return peak_normalize(x, 0.9).astype(np.float64), "IR fragment"


def gen_image_scanline(img_gray, gen_sr, micro_ms, seed):
    """One random image row, zero-mean, stretched to n, Hann, exp-smoothed (MS:350-362)."""
    rng = np.random.default_rng(int(seed))
    n = grain_len(gen_sr, micro_ms, 64)
    if img_gray is None:
        return np.zeros(n, dtype=np.float64), "No image loaded"
    h, w = img_gray.shape
    y = int(rng.integers(0, h))
    line = img_gray[y, :].astype(np.float64) / 255.0
    line = (line - line.mean()) * 2.0
    x = np.interp(np.linspace(0, 1, n), np.linspace(0, 1, w), line)
    x *= hann(n)
    x = np.convolve(x, np.exp(-np.linspace(0, 5, 48)), mode="same")
    return x.astype(np.float64), f"Image line y={y}"


# ---------------------------------------------------------------------------
# Physical-ish models (MS:369-402)
# ---------------------------------------------------------------------------
def resonator_bank(x, sr, modes=24, f_min=120, f_max=12000, decay_ms=80, seed=0):
    """Log-spaced decaying sinusoid bank mixed by sign(x) (MS:369-384)."""
    rng = np.random.default_rng(int(seed) + 321)
    n = len(x)
    if n < 32:
        return x
    t = np.arange(n, dtype=np.float64) / sr
    env = np.exp(-t / max(1e-6, decay_ms / 1000.0))
    acc = np.zeros_like(x)
    m = int(max(1, modes))
    for k in range(m):
        f = float(f_min) * ((float(f_max) / max(1.0, float(f_min))) ** (k / max(1, m - 1)))
        f *= 2.0 ** rng.uniform(-0.02, 0.02)
        ph = rng.uniform(0, 2 * np.pi)
        acc += (1.0 / (1 + k * 0.35)) * np.sin(2 * np.pi * f * t + ph) * env
    acc = acc / max(1e-12, np.max(np.abs(acc)))
    return (0.55 * x + 0.45 * (x * 0.0 + acc) * np.sign(x)).astype(np.float64)


def waveguide_splinters(x, sr, lines=8, max_ms=8.0, feedback=0.7, seed=0):
    """Cascade of recursive comb lines applied in place (MS:386-402)."""
    rng = np.random.default_rng(int(seed) + 777)
    n = len(x)
    if n < 64:
        return x
    y = x.copy()
    for _ in range(int(max(1, lines))):
        d = int(max(1, round((rng.uniform(0.4, max_ms) / 1000.0) * sr)))
        g = feedback * rng.uniform(0.6, 0.98)
        mix = rng.uniform(0.15, 0.45)
        buf = np.zeros(d, dtype=np.float64)
        wp = 0
        for t in range(n):
            v = y[t] + g * buf[wp]
            buf[wp] = v
            wp = (wp + 1) % d
            y[t] = (1.0 - mix) * y[t] + mix * v
    return y.astype(np.float64)


# ---------------------------------------------------------------------------
# Space (MS:409-445)
# ---------------------------------------------------------------------------
def er_taps(sr, taps=320, max_ms=45, seed=0):
    """Early-reflection tap table (offset samples, gain) drawn from seed+202 (MS:410-417)."""
    rng = np.random.default_rng(int(seed) + 202)
    delays = rng.uniform(0.3, max_ms, size=int(max(1, taps))) / 1000.0
    gains = rng.uniform(-1.0, 1.0, size=delays.size)
    gains *= np.exp(-delays * 42.0)
    offs = np.array([int(round(d * sr)) for d in delays], dtype=np.int64)
    return offs, gains


def early_reflection_cloud(x, sr, taps=320, max_ms=45, seed=0):
    """Identity + sparse FIR over the dry input, in tap order (MS:409-421)."""
    offs, gains = er_taps(sr, taps, max_ms, seed)
    n = len(x)
    y = x.copy()
    for off, g in zip(offs, gains):
        if 0 < off < n:
            y[off:] += g * x[:-off]
    return y.astype(np.float64)


def stereo_shifts(sr, width):
    """Left/right circular shifts in samples (MS:428-429)."""
    w = float(np.clip(width, 0.0, 1.0))
    return int(round((1 + 7 * w) * 0.0005 * sr)), int(round((1 + 9 * w) * 0.0007 * sr))


def spectral_diffusion_stereo(x, sr, width=0.6):
    """L = roll(x, dl); R = phase-rotated roll(x, -dr) (MS:423-436)."""
    w = float(np.clip(width, 0.0, 1.0))
    n = len(x)
    if n < 64:
        return np.column_stack([x, x])
    dl, dr = stereo_shifts(sr, w)
    L = np.roll(x, dl)
    X = np.fft.rfft(np.roll(x, -dr))
    k = np.arange(X.size, dtype=np.float64)
    rot = np.exp(1j * (w * 0.9) * np.sin(2 * np.pi * k / max(1.0, k[-1])))
    return np.column_stack([L, np.fft.irfft(X * rot, n=n)]).astype(np.float64)


def ir_kernel(ir):
    """Mono, <= 8192 taps (MS:439-443); None when absent or shorter than 8."""
    if ir is None or ir.size < 8:
        return None
    h = ir.astype(np.float64)
    if h.ndim > 1:
        h = h.mean(axis=1)
    return h[:min(h.size, IR_TAP_CAP)]


def convolve_ir_short(x, ir):
    """Causal direct FIR, first len(x) samples of the full convolution (MS:438-445)."""
    h = ir_kernel(ir)
    if h is None:
        return x
    return np.convolve(x, h, mode="full")[:len(x)].astype(np.float64)


def fir_causal(x, h):
    """The arithmetic of MS:444 without the 8192-tap cap of MS:443: the standalone
    FIR of SURVEY §8 (16 k / 64 k taps), np.convolve(x, h)[:len(x)] in float64."""
    x = np.asarray(x, dtype=np.float64)
    return np.convolve(x, np.asarray(h, dtype=np.float64), mode="full")[:len(x)]


def synthetic_fir_taps(M, seed=7):
    """SURVEY §8(d)'s standalone-FIR taps: default_rng(7).standard_normal(M) exp(-6t/M), peak 0.9."""
    h = np.random.default_rng(seed).standard_normal(M) * np.exp(-6.0 * np.arange(M) / M)
    return peak_normalize(h, 0.9)


# ---------------------------------------------------------------------------
# Breakpoint lanes (MS:452-482), unfold (MS:489-500), event fields (MS:507-558)
# ---------------------------------------------------------------------------
def parse_breakpoints(s):
    """"t:v, t:v" -> sorted [(t, v)]; malformed parts skipped, "a:b:c" raises (MS:452-467)."""
    pts = []
    s = (s or "").strip()
    if not s:
        return pts
    for part in s.split(","):
        part = part.strip()
        if not part or ":" not in part:
            continue
        t, v = part.split(":")
        try:
            pts.append((float(t.strip()), float(v.strip())))
        except Exception:
            pass
    pts.sort(key=lambda p: p[0])
    return pts


def eval_breakpoints(pts, t, default):
    """Piecewise-linear lane, held at both ends (MS:469-482)."""
    if not pts:
        return default
    if t <= pts[0][0]:
        return pts[0][1]
    if t >= pts[-1][0]:
        return pts[-1][1]
    for (t0, v0), (t1, v1) in zip(pts[:-1], pts[1:]):
        if t0 <= t <= t1:
            a = (t - t0) / max(1e-12, (t1 - t0))
            return (1 - a) * v0 + a * v1
    return default


def unfold_multiband(x_gen, gen_sr, bands_out_hz, unfolds, roll_hz=0.0):
    """Sum of band-passes with edges scaled by each band's unfold (MS:492-500)."""
    out = None
    for (lo, hi), u in zip(bands_out_hz, unfolds):
        y = bandpass_fft(x_gen, gen_sr, lo * u, hi * u, roll=roll_hz).astype(np.float64, copy=False)
        out = y if out is None else (out + y)
    return out if out is not None else x_gen


def generate_event_times(process, dur_s, rate, seed, cluster_size=6, cluster_spread_ms=25,
                         hawkes_gain=0.6, hawkes_decay_s=0.25):
    """Event onsets in seconds from default_rng(seed+9999) (MS:507-558)."""
    rng = np.random.default_rng(int(seed) + 9999)
    if process == "Single" or rate <= 0:
        return [0.0]
    times = []
    if process == "Poisson":                              # MS:518-524
        t = 0.0
        while t < dur_s:
            t += rng.exponential(1.0 / rate)
            if t < dur_s:
                times.append(t)
    elif process == "Clustered":                          # MS:526-542
        parents, t = [], 0.0
        prate = max(0.1, rate / max(1, cluster_size))
        while t < dur_s:
            t += rng.exponential(1.0 / prate)
            if t < dur_s:
                parents.append(t)
        spread = cluster_spread_ms / 1000.0
        for p in parents:
            k = int(max(1, round(rng.uniform(0.6, 1.4) * cluster_size)))
            for _ in range(k):
                tt = p + rng.normal(0.0, spread)
                if 0.0 <= tt < dur_s:
                    times.append(tt)
        times.sort()
    elif process == "Hawkes":                             # MS:544-556
        dt = 0.002
        act = 0.0
        for i in range(int(math.ceil(dur_s / dt))):
            t = i * dt
            act *= math.exp(-dt / max(1e-6, hawkes_decay_s))
            lam = rate + hawkes_gain * act * rate
            if rng.random() < min(0.95, lam * dt):
                times.append(t + rng.uniform(0, dt))
                act += 1.0
    return times


class SpectralImprint:
    """EMA of grain magnitudes re-imposed on later grains (MS:565-581)."""

    def __init__(self):
        self.mem = None

    def apply(self, x, amount=0.35, smooth=0.92):
        n = len(x)
        if n < 64 or amount <= 0:
            return x
        X = np.fft.rfft(x)
        mag = np.abs(X)
        if self.mem is None or self.mem.size != mag.size:
            self.mem = mag.copy()
        else:
            self.mem = smooth * self.mem + (1.0 - smooth) * mag
        Y = ((1.0 - amount) * mag + amount * self.mem) * np.exp(1j * np.angle(X))
        return np.fft.irfft(Y, n=n).astype(np.float64)


# ---------------------------------------------------------------------------
# Render: plan -> grains -> output stage (MS:588-792)
# ---------------------------------------------------------------------------
@dataclass
class EventPlan:
    index: int            # i in the reference loop (seed+i for generators)
    t0: float
    amp: float
    ufac: float
    gen_sr: int
    n: int
    cutoff_out: float
    stretch: float
    start: int            # output sample; events with start >= out_n are not placed
    offset: int           # read offset into the grain (MS:746-751)
    placed: bool


@dataclass
class RenderPlan:
    base_sr: int
    out_n: int
    gen_sr: int
    events: list = field(default_factory=list)


def design_sr(base_sr: int, unfold: float) -> int:
    """clip(round(base_sr*unfold), base_sr, 30 MHz) (MS:596-597, 645-646)."""
    return int(np.clip(int(round(base_sr * unfold)), base_sr, GEN_SR_CAP))


def event_grain_len(p: dict, gen_sr: int) -> int:
    """Length every grain keeps through the chain, by generator mode (MS:650-686)."""
    mode = p["gen_mode"]
    micro_ms = float(p["micro_ms"])
    if mode == "Crackle / corona":
        # np.convolve(x, ker, "same") is max(len(x), len(ker)) long (MS:280-281)
        return max(grain_len(gen_sr, micro_ms), max(8, int(p["crackle_kernel"])))
    if mode in BASIC_MODES:
        return grain_len(gen_sr, micro_ms)
    if mode in ("Stick–slip friction", "Micro-chaos", "Image scanline"):
        return grain_len(gen_sr, micro_ms, 64)
    if mode == "Wavelet atoms":
        return grain_len(gen_sr, micro_ms, 128)
    if mode == "IR fragment":
        ir = p.get("_ir_audio")
        return grain_len(gen_sr, micro_ms, 16 if (ir is None or ir.size < 32) else 64)
    return grain_len(gen_sr, micro_ms)   # MS:686 fallback: Noise burst


def plan_render(p: dict) -> RenderPlan:
    """All scalar and RNG decisions of a render, before any synthesis (MS:589-646, 742-751).

    The per-render stream ``default_rng(seed+123456)`` draws one uniform per event
    (amp, MS:642) and, only for placed events, one bounded integer (offset,
    MS:746-751), interleaved in event order.  Grain sizes never change through
    the chain, so offsets can be drawn before synthesis.
    """
    base_sr = int(p["base_sr"])
    out_dur = float(p["out_dur_s"])
    out_n = int(max(1, round(out_dur * base_sr)))
    unfold0 = max(1.0, float(p["time_unfold"]))
    plan = RenderPlan(base_sr, out_n, design_sr(base_sr, unfold0))
    lanes = [parse_breakpoints(p[k]) for k in ("bp_density", "bp_unfold", "bp_cutoff", "bp_stretch")]
    rate = float(p["grains_per_sec"])
    times = generate_event_times(p["event_process"], out_dur, rate, seed=int(p["seed"]),
                                 cluster_size=int(p["cluster_size"]),
                                 cluster_spread_ms=float(p["cluster_spread_ms"]),
                                 hawkes_gain=float(p["hawkes_gain"]),
                                 hawkes_decay_s=float(p["hawkes_decay_s"]))[:int(p["max_grains"])]
    rng = np.random.default_rng(int(p["seed"]) + 123456)
    ar = float(p["grain_amp_rand"])
    max_off = int(round((float(p["grain_offset_max_ms"]) / 1000.0) * base_sr))
    for i, t0 in enumerate(times):
        dens = eval_breakpoints(lanes[0], t0, default=rate)
        ufac = eval_breakpoints(lanes[1], t0, default=unfold0)
        cut = eval_breakpoints(lanes[2], t0, default=float(p["bandlimit_out_hz"]))
        st = eval_breakpoints(lanes[3], t0, default=float(p["partial_stretch"]))
        amp = 1.0
        if rate > 0:
            amp *= np.clip(dens / max(1e-6, rate), 0.15, 4.0)
        amp *= rng.uniform(1.0 - ar, 1.0 + ar)
        ufac = max(1.0, float(ufac))
        gsr = design_sr(base_sr, ufac)
        n = event_grain_len(p, gsr)
        start = int(round(t0 * base_sr))
        placed = start < out_n
        offset = 0
        if placed and p["grain_offset_on"] and max_off > 0:
            offset = int(rng.integers(0, max(1, min(max_off, n))))
        plan.events.append(EventPlan(i, t0, float(amp), ufac, gsr, n, float(cut), float(st),
                                     start, offset, placed))
    return plan


def synth_micro(p: dict, ev: EventPlan):
    """Generator dispatch for event ev -> (x, note) (MS:650-686)."""
    mode = p["gen_mode"]
    s = int(p["seed"]) + ev.index
    g = ev.gen_sr
    mm = float(p["micro_ms"])
    if mode in BASIC_MODES:
        return gen_basic(g, mm, s, mode, float(p["dust_density"]), float(p["noise_tilt"]),
                         float(p["ring_hz"]), float(p["ring_decay_ms"])), ""
    if mode == "Crackle / corona":
        return gen_crackle(g, mm, s, float(p["crackle_alpha"]), float(p["crackle_density"]),
                           int(p["crackle_kernel"])), ""
    if mode == "Stick–slip friction":
        return gen_stick_slip(g, mm, s, float(p["ss_threshold"]), float(p["ss_build"]),
                              float(p["ss_decay"]), float(p["ss_noise"])), ""
    if mode == "Micro-chaos":
        return gen_micro_chaos(g, mm, s, float(p["chaos_r"]), float(p["chaos_gate"])), ""
    if mode == "Wavelet atoms":
        return gen_wavelet_atoms(g, mm, s, float(p["wav_base_hz"]), int(p["wav_count"]),
                                 float(p["wav_spread"])), ""
    if mode == "IR fragment":
        return gen_ir_fragment(p.get("_ir_audio"), g, mm, s)
    if mode == "Image scanline":
        return gen_image_scanline(p.get("_img_gray"), g, mm, s)
    return gen_basic(g, mm, s, "Noise burst", 0.01, -3.0, 4000, 12), ""


def spectral_chain(p: dict, ev: EventPlan, xg: np.ndarray) -> np.ndarray:
    """Band-limit -> warps -> stretch -> physics -> unfold for one grain (MS:690-727)."""
    g = ev.gen_sr
    if p["bandlimit_on"]:
        xg = lowpass_fft(xg, g, ev.cutoff_out * ev.ufac, roll=float(p["bandlimit_roll_hz"]))
    if p["nl_warp_on"]:
        xg = fft_warp_power(xg, float(p["nl_warp_power"]))
    if p["cep_warp_on"]:
        xg = cepstral_warp(xg, float(p["cep_factor"]))
    if p["partial_lock_on"]:
        xg = partial_lock_stretch(xg, ev.stretch, top_n=int(p["pl_top_n"]),
                                  neighborhood=int(p["pl_neigh"]))
    else:
        xg = fft_partial_stretch(xg, ev.stretch)
    s = int(p["seed"]) + ev.index
    if p["res_bank_on"]:
        xg = resonator_bank(xg, g, int(p["res_modes"]), float(p["res_fmin"]),
                            float(p["res_fmax"]), float(p["res_decay_ms"]), s)
    if p["wg_on"]:
        xg = waveguide_splinters(xg, g, int(p["wg_lines"]), float(p["wg_max_ms"]),
                                 float(p["wg_fb"]), s)
    if p["unfold_mode"] == "Classic reinterpret":
        return xg.astype(np.float64, copy=False)             # MS:489-490 identity
    bands = [(0, float(p["mb_b1"])), (float(p["mb_b1"]), float(p["mb_b2"])),
             (float(p["mb_b2"]), float(p["mb_b3"]))]
    us = [float(p["mb_u1"]), float(p["mb_u2"]), float(p["mb_u3"])]
    return unfold_multiband(xg, g, bands, us, roll_hz=float(p["mb_roll"]))


def output_stage(p: dict, mono: np.ndarray, base_sr: int) -> np.ndarray:
    """ADSR -> ER -> IR -> stereo -> tanh -> normalise (MS:760-781)."""
    out_n = mono.size
    mono = mono * make_adsr(out_n, base_sr, float(p["env_a"]), float(p["env_d"]),
                            float(p["env_s"]), float(p["env_r"]), float(p["env_curve"]))
    if p["er_cloud_on"]:
        mono = early_reflection_cloud(mono, base_sr, taps=int(p["er_taps"]),
                                      max_ms=float(p["er_max_ms"]), seed=int(p["seed"]))
    if p["space_ir_on"] and p.get("_ir_audio") is not None:
        mono = convolve_ir_short(mono, p["_ir_audio"][:int(p["space_ir_max_samps"])])
    if p["stereo_on"]:
        st = spectral_diffusion_stereo(mono, base_sr, width=float(p["stereo_width"]))
    else:
        st = np.column_stack([mono, mono])
    st = tanh_clip(st, drive=float(p["sat_drive"]))
    return peak_normalize(st, peak=float(p["peak"]))


def render(p: dict, progress=None):
    """Reference-equivalent render: (float64 (out_n, 2), meta) (MS:588-792)."""
    plan = plan_render(p)
    if progress:
        progress(0, f"Output SR {plan.base_sr} Hz | Design SR {plan.gen_sr} Hz")
    out = np.zeros(plan.out_n, dtype=np.float64)
    imprint = SpectralImprint() if p["spectral_imprint_on"] else None
    prev = None
    micro_last = grain_last = None
    nev = len(plan.events)
    for ev in plan.events:
        xg, note = synth_micro(p, ev)
        micro_last = xg.copy()
        grain = spectral_chain(p, ev, xg)
        grain_last = grain.copy()
        if p["event_feedback_on"] and prev is not None:        # MS:731-734
            fb = float(p["event_feedback_amt"])
            L = min(len(grain), len(prev))
            grain[:L] = (1.0 - fb) * grain[:L] + fb * prev[:L]
        if imprint is not None:                                # MS:736-738
            grain = imprint.apply(grain, amount=float(p["spectral_imprint_amt"]),
                                  smooth=float(p["spectral_imprint_smooth"]))
        prev = grain.copy()
        if not ev.placed:
            continue
        g = grain[ev.offset:]
        L = min(plan.out_n - ev.start, g.size)
        if L > 0:
            out[ev.start:ev.start + L] += ev.amp * g[:L]
        if progress and (ev.index % 50 == 0):
            progress(int(5 + 70 * (ev.index / max(1, nev))), f"Events {ev.index}/{nev}  {note}".strip())
    st = output_stage(p, out, plan.base_sr)
    if progress:
        progress(100, "Done.")
    meta = {"out_sr": plan.base_sr, "design_sr_base": plan.gen_sr,
            "micro_last": micro_last, "grain_last": grain_last}
    return st.astype(np.float64), meta


# ---------------------------------------------------------------------------
# UI analysis helpers (MS:23-24, 197-212): the spectrogram the app draws
# ---------------------------------------------------------------------------
def db(x, eps=1e-12):
    """20 log10(max(|x|, eps)) (MS:23-24)."""
    return 20 * np.log10(np.maximum(np.abs(x), eps))


def stft_mag_db(x, sr, win=2048, hop=256, max_frames=3000):
    """Hann-windowed STFT magnitude in dB, (win//2+1, frames) (MS:197-212)."""
    n = len(x)
    if n < win:
        X = np.fft.rfft(x * hann(n), n=win)
        return db(X)[:, None]
    frames = min(1 + (n - win) // hop, max_frames)
    w = hann(win)
    S = np.empty((win // 2 + 1, frames), dtype=np.float64)
    for i in range(frames):
        a = i * hop
        S[:, i] = db(np.fft.rfft(x[a:a + win] * w))
    return S
