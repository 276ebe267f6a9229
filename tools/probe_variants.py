#!/usr/bin/env python3
"""Debug probe (GPU box): device vs oracle for variants of one shipped preset,
next to the oracle's own float64 rounding spread (FFT evaluated as F(3x)/3).

    python tools/probe_variants.py PRESET key=value[,key=value] ...
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

import msgpu  # noqa: E402
from oracle import msound_oracle as O  # noqa: E402


def rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)))


def main():
    info = json.load(open(os.path.join(REPO, "tests", "golden", "golden_info.json")))
    full = np.load(os.path.join(REPO, "tests", "golden", "render_full.npz"))
    irs = np.load(os.path.join(REPO, "tests", "golden", "irs.npz"))
    name = sys.argv[1]
    variants = [""] + sys.argv[2:]
    for v in variants:
        p = msgpu.merged(info["preset_params"][name])
        p["out_dur_s"] = 0.5
        p["_ir_audio"] = irs["tiny_room_ir"]
        p["_img_gray"] = full["image_gray"]
        for kv in filter(None, v.split(",")):
            k, val = kv.split("=")
            old = p[k]
            p[k] = type(old)(val) if not isinstance(old, bool) else val in ("1", "True", "true")
        a, _ = msgpu.render(p)
        ref, _ = O.render(p)
        r0, i0 = np.fft.rfft, np.fft.irfft
        np.fft.rfft = lambda x, n=None: r0(np.asarray(x) * 3.0, n=n) / 3.0
        np.fft.irfft = lambda X, n=None: i0(np.asarray(X) * 3.0, n=n) / 3.0
        alt, _ = O.render(p)
        np.fft.rfft, np.fft.irfft = r0, i0
        print(f"{name} [{v or 'as shipped'}]: device-oracle {rms(a, ref):.3e}  oracle spread {rms(alt, ref):.3e}",
              flush=True)


if __name__ == "__main__":
    main()
