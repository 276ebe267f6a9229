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


def render_batch(params_list, device: int = 0):
    from .dropin import render_batch as _rb
    return _rb(params_list, device)
