"""The app's batch render (``AudioApp.on_batch``, MS:1524-1596) on the device.

The reference loops seeds x base-unfold x stretch-factor (outer to inner),
renders each variant with ``render(p)`` and writes it with
``sf.write(path, audio.astype(np.float32), out_sr)``.  Here the whole triple
product goes to the device as batches of presets (``render_batch``; one
workgroup grid per batch, no per-variant launch sequence) and each variant is
written as a float32 WAV by a small RIFF writer (soundfile is not a
dependency).

File names: the reference builds
``f"ms_seed{sd}_unf{u:g}_st{st:g}_{out_sr}Hz.wav".replace(".", "p")`` (MS:1587),
which also turns the ``.wav`` suffix into ``pwav``; libsndfile then cannot infer
a format from that name and the reference's batch stops at its first file.
``names="reference"`` keeps that exact string (the writer here does not need
an extension); the default ``names="wav"`` applies the same replacement to the
stem and keeps a real ``.wav`` suffix.
"""
from __future__ import annotations

import os
import struct

import numpy as np

from .params import merged

# presets per device batch: bounds the output buffer (frames x 2 float32) and
# the per-batch event tables; the batch scheduler handles any mix of lengths.
MAX_BATCH_PRESETS = 1024
MAX_BATCH_FRAMES = 1 << 30      # 8 GiB of float32 stereo output


def parse_list(s, cast=float):
    """Comma-separated list, unparsable entries skipped (MS:1557-1566)."""
    out = []
    for p in str(s).split(","):
        p = p.strip()
        if not p:
            continue
        try:
            out.append(cast(p))
        except Exception:
            pass
    return out


def variant_name(sd, u, st, out_sr, names="wav"):
    if names == "reference":
        return f"ms_seed{sd}_unf{u:g}_st{st:g}_{out_sr}Hz.wav".replace(".", "p")
    if names == "wav":
        return f"ms_seed{sd}_unf{u:g}_st{st:g}_{out_sr}Hz".replace(".", "p") + ".wav"
    raise ValueError("names must be 'wav' or 'reference'")


def variants(base_params, seeds, unfolds, stretches):
    """The parameter dicts in the reference's loop order (MS:1580-1586)."""
    if isinstance(seeds, str):
        seeds = parse_list(seeds, int)
    if isinstance(unfolds, str):
        unfolds = parse_list(unfolds, float)
    if isinstance(stretches, str):
        stretches = parse_list(stretches, float)
    out = []
    for sd in seeds:
        for u in unfolds:
            for st in stretches:
                p = dict(base_params)
                p["seed"] = int(sd)
                p["time_unfold"] = float(u)
                p["partial_stretch"] = float(st)
                out.append(((sd, u, st), p))
    return out


def write_wav_float32(path, audio, sr):
    """IEEE-float WAV (format tag 3, fmt + fact + data chunks), frames x channels."""
    a = np.ascontiguousarray(audio, dtype="<f4")
    if a.ndim == 1:
        a = a[:, None]
    frames, ch = a.shape
    data_bytes = a.nbytes
    if data_bytes + 64 > 0xFFFFFFFF:
        raise ValueError("WAV data beyond 4 GiB")
    fmt = struct.pack("<HHIIHHH", 3, ch, int(sr), int(sr) * ch * 4, ch * 4, 32, 0)
    fact = struct.pack("<I", frames)
    riff_size = 4 + (8 + len(fmt)) + (8 + len(fact)) + (8 + data_bytes)
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", riff_size) + b"WAVE")
        f.write(b"fmt " + struct.pack("<I", len(fmt)) + fmt)
        f.write(b"fact" + struct.pack("<I", len(fact)) + fact)
        f.write(b"data" + struct.pack("<I", data_bytes))
        a.tofile(f)


def read_wav_float32(path):
    """Reader for the files write_wav_float32 makes: (frames x channels float32, sr)."""
    with open(path, "rb") as f:
        b = f.read()
    if b[:4] != b"RIFF" or b[8:12] != b"WAVE":
        raise ValueError("not a RIFF/WAVE file")
    pos, ch, sr, data = 12, None, None, None
    while pos + 8 <= len(b):
        tag, size = b[pos:pos + 4], struct.unpack("<I", b[pos + 4:pos + 8])[0]
        body = b[pos + 8:pos + 8 + size]
        if tag == b"fmt ":
            tagv, ch, sr = struct.unpack("<HHI", body[:8])
            if tagv != 3:
                raise ValueError("not an IEEE-float WAV")
        elif tag == b"data":
            data = np.frombuffer(body, dtype="<f4")
        pos += 8 + size + (size & 1)
    if ch is None or data is None:
        raise ValueError("missing fmt or data chunk")
    return data.reshape(-1, ch).copy(), sr


def _chunks(items, frames_of):
    cur, tot = [], 0
    for it in items:
        fr = frames_of(it)
        if cur and (len(cur) >= MAX_BATCH_PRESETS or tot + fr > MAX_BATCH_FRAMES):
            yield cur
            cur, tot = [], 0
        cur.append(it)
        tot += fr
    if cur:
        yield cur


def render_variations(base_params, seeds, unfolds, stretches, folder=None, device: int = 0,
                      names="wav", progress=None, devices=None):
    """Render every (seed, unfold, stretch) variant of ``base_params`` on the device
    (or, with ``devices``, sharded across those GPUs, multi.py).

    Returns a list of ``(name, audio, out_sr)`` in the reference's order (audio
    (out_n, 2) float32); with ``folder``, also writes each as a float32 WAV.
    ``progress(percent, text)`` gets the reference's status line per file.
    """
    from .pack import PackedBatch, out_frames

    base = merged(base_params)
    pairs = variants(base, seeds, unfolds, stretches)
    keys = [key for key, _ in pairs]
    total = max(1, len(keys))
    out_sr = int(base["base_sr"])                 # every variant has the template's out_n and out_sr
    results = []

    def emit(key, audio):
        name = variant_name(*key, out_sr, names)
        if folder is not None:
            write_wav_float32(os.path.join(folder, name), audio, out_sr)
        results.append((name, audio, out_sr))
        if progress:
            progress(int(100 * len(results) / total), f"Batch: {len(results)}/{total} → {name}")

    if devices is not None and len(list(devices)) > 1:
        from .multi import pool_for
        for key, audio in zip(keys, pool_for(devices).render_batch([p for _, p in pairs])):
            emit(key, audio)
        return results
    if devices is not None:
        device = int(list(devices)[0])
    from .engine import default_engine
    eng = default_engine(device)
    frames = out_frames(base)
    for chunk in _chunks(keys, lambda k: frames):
        packed = PackedBatch.variants(base, chunk)   # the template packed once (MS:1578-1584)
        out = eng.render_packed(packed)
        eng.torch.cuda.synchronize(eng.device)
        host = out.cpu().numpy()
        for key, off, n in zip(chunk, packed.offsets, packed.out_n):
            emit(key, host[off:off + n].copy())
    return results
