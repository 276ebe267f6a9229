"""Drop-in ``render(params, progress=None)`` for microsound_0.2.1/main_v2.py:588.

Usage from the unchanged PyQt6 front-end::

    import main_v2, msgpu
    main_v2.render = msgpu.render      # RenderWorker.run (MS:811) and on_batch (MS:1585)

Returns ``(audio, meta)`` like the reference: ``audio`` is a C-contiguous
(out_n, 2) float32 array (the consumers only read its shape/columns and cast
with ``astype(np.float32)`` before ``sf.write``, MS:1473-1519, 1589), ``meta``
has ``out_sr``, ``design_sr_base``, ``micro_last``, ``grain_last`` (MS:786-791).
The ``progress`` callback gets the reference's messages: 0 with the SR line,
every 50th event, and 100 "Done." (MS:599-600, 757-758, 783-784).  The event
messages are sent from the render's plan while the device is still rendering
(msg_render_batch returns once the batch is enqueued), "Done." after the
device has finished.

Errors follow the reference: ``KeyError`` for a key ``render`` indexes and the
dict lacks (pass ``msgpu.merged(partial)`` for a partial preset, as the UI's
loader merges it over the factory defaults), ``ValueError`` where MS raises it,
``NotImplementedError`` for the device limits in DESIGN.md.
"""
from __future__ import annotations

import numpy as np

from .engine import default_engine
from .pack import PackedBatch, design_sr
from .params import first_missing_key, merged

def render(params, progress=None, device: int = 0):
    missing = first_missing_key(params)
    if missing is not None:
        raise KeyError(missing)
    p = merged(params)
    base_sr = int(p["base_sr"])
    if progress:
        progress(0, f"Output SR {base_sr} Hz | Design SR {design_sr(p)} Hz")
    eng = default_engine(device)
    packed = PackedBatch([p])
    out = eng.render_packed(packed)           # returns once enqueued
    info = eng.last_plan()[0]
    if progress:                              # MS:757-758, while the device renders
        events = eng.last_events(0)
        n = len(events)
        for e in events:
            if e.len > 0 and e.index % 50 == 0:
                note = _event_note(p, e.index)
                progress(int(5 + 70 * (e.index / max(1, n))), f"Events {e.index}/{n}  {note}".strip())
    eng.torch.cuda.synchronize(eng.device)
    audio = out.cpu().numpy().reshape(packed.total_frames, 2)
    if progress:
        progress(100, "Done.")
    micro = grain = None
    if info.n_events > 0:
        micro, grain = eng.last_meta(0, int(info.max_n))
    meta = {"out_sr": base_sr, "design_sr_base": int(info.design_sr),
            "micro_last": micro, "grain_last": grain}
    return np.ascontiguousarray(audio), meta


def _event_note(p, i):
    """The generator note of event i (MS:342-362, shown by MS:758): "IR fragment",
    "Image line y=<row>" with the row drawn by default_rng(seed + i).integers(0, h)
    (the library's NumPy-exact stream, msg_rng_integers), or the no-source notes."""
    mode = p["gen_mode"]
    if mode == "IR fragment":
        ir = p.get("_ir_audio")
        return "No IR loaded" if (ir is None or np.asarray(ir).size < 32) else "IR fragment"
    if mode == "Image scanline":
        img = p.get("_img_gray")
        if img is None:
            return "No image loaded"
        from . import _lib as L
        import ctypes as C
        y = C.c_int64(0)
        L.check(L.lib().msg_rng_integers(int(p["seed"]) + int(i), 0, int(np.asarray(img).shape[0]), C.byref(y), 1),
                None)
        return f"Image line y={y.value}"
    return ""


def render_batch(params_list, device: int = 0, results: str = "audio"):
    """Render many presets in one device batch; returns a list of (out_n, 2) float32
    arrays ("audio"), per-preset summaries ("stats", multi.rec_stats's fields,
    reduced on the device by msg_digest) or the device tensors themselves ("device")."""
    if results not in ("audio", "stats", "device"):
        raise ValueError("results must be 'audio', 'stats' or 'device'")
    eng = default_engine(device)
    packed = PackedBatch(list(params_list))
    out = eng.render_packed(packed)
    if results == "device":
        return [out[int(o):int(o) + int(n)] for o, n in zip(packed.offsets, packed.out_n)]
    eng.torch.cuda.synchronize(eng.device)
    if results == "stats":
        from .multi import device_stats
        return device_stats(eng, out, packed.offsets, packed.out_n)
    host = out.cpu().numpy()
    return [host[o:o + n].copy() for o, n in zip(packed.offsets, packed.out_n)]
