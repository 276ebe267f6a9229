"""msgpu — MI355X-native Microsound render engine.

Drop-in for ``microsound_0.2.1/main_v2.py:render``::

    import msgpu
    audio, meta = msgpu.render(params)           # same signature as the reference

The compute path is libmsgpu.so (HIP kernels for gfx950) bound by ctypes; there
is no CPU fallback.
"""
from .params import DEFAULTS, CONFIGS, config_params, merged  # noqa: F401


def render(params, progress=None, device: int = 0):
    from .dropin import render as _render
    return _render(params, progress, device)


def render_batch(params_list, device: int = 0, devices=None, results: str = "audio"):
    """Render many presets; ``devices`` (e.g. range(8)) shards them across GPUs,
    one worker process per GPU (multi.py; call before this process touches the GPU).
    ``results``: "audio" ((out_n, 2) float32 arrays), "stats" (a summary per
    preset, multi.audio_stats) or "device" (the renders stay in HBM: device
    tensors on one GPU, multi.DeviceResult handles across several)."""
    if devices is not None and len(list(devices)) > 1:
        from .multi import pool_for
        return pool_for(devices).render_batch(params_list, results=results)
    if devices is not None:
        device = int(list(devices)[0])
    from .dropin import render_batch as _rb
    return _rb(params_list, device, results)


def DevicePool(devices, stub: bool = False, share_devices: bool = False):
    """One render worker per GPU (multi.py); create it before any GPU call."""
    from .multi import DevicePool as _P
    return _P(devices, stub, share_devices)


def stft_mag_db(x, sr=None, win=2048, hop=256, max_frames=3000, device: int = 0):
    """The app's spectrogram (MS:197-212) on the device; see spectrum.py."""
    from .spectrum import stft_mag_db as _s
    return _s(x, sr, win, hop, max_frames, device)


def fir(x, h, device: int = 0):
    """Standalone causal FIR np.convolve(x, h)[:len(x)] on the device (MS:444 arithmetic, any tap count)."""
    from .engine import default_engine
    import numpy as np
    eng = default_engine(device)
    torch = eng.torch
    if isinstance(x, torch.Tensor):
        return eng.fir(x.contiguous(), h)[0]
    a = np.ascontiguousarray(x, dtype=np.float32)
    y, _ = eng.fir(torch.from_numpy(a).to(f"cuda:{eng.device}"), h)
    torch.cuda.synchronize(eng.device)
    return y.cpu().numpy()


def render_variations(base_params, seeds, unfolds, stretches, folder=None, device: int = 0, devices=None, **kw):
    """The app's batch render (on_batch, MS:1524-1596); see batch.py.  ``devices``
    shards the variants across GPUs as render_batch does."""
    from .batch import render_variations as _rv
    return _rv(base_params, seeds, unfolds, stretches, folder, device, devices=devices, **kw)
