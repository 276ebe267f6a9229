"""The app's analysis view on the device: ``stft_mag_db`` (MS:197-212).

``AudioApp.update_plots`` (MS:1498-1500) shows ``stft_mag_db(y.mean(axis=1), sr,
win, hop)`` with win/hop 2048/256 below 96 kHz and 4096/512 from 96 kHz up.
Each frame is one workgroup of the float64 FFT engine (``k_stft64``), so the
result matches NumPy's pocketfft to float64 rounding.  Bins whose magnitude
sits at the float64 noise floor (|X| ~ 1e-13 relative) differ in dB between
any two FFT implementations; tests compare the rest exactly (tests/
test_gpu_spectrum.py).
"""
from __future__ import annotations

import numpy as np

from .engine import default_engine


def display_stft_params(sr: int):
    """win, hop used by update_plots (MS:1498-1499)."""
    return (2048, 256) if sr < 96000 else (4096, 512)


def stft_mag_db(x, sr=None, win=2048, hop=256, max_frames=3000, device: int = 0):
    """S (win//2 + 1, frames) float64 in dB, like the reference.

    ``x``: mono (n,) or stereo (n, 2) samples, a NumPy array or a float32 device
    tensor (e.g. the output of ``Engine.render_packed``); stereo is analysed as
    the L/R mean, as MS:1500 does.  ``sr`` is unused, as in the reference.
    A device tensor returns a device tensor; a NumPy input returns NumPy.
    """
    eng = default_engine(device)
    torch = eng.torch
    on_device = isinstance(x, torch.Tensor)
    if on_device:
        xd = x if x.dtype in (torch.float32, torch.float64) else x.to(torch.float64)
        xd = xd.contiguous()
    else:
        a = np.asarray(x)
        a = np.ascontiguousarray(a, dtype=np.float32 if a.dtype == np.float32 else np.float64)
        xd = torch.from_numpy(a).to(f"cuda:{eng.device}")
    S = eng.stft_mag_db(xd, win, hop, max_frames)
    if on_device:
        return S.t()
    torch.cuda.synchronize(eng.device)
    return np.ascontiguousarray(S.cpu().numpy().T)
