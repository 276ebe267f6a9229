#!/usr/bin/env python3
"""Golden vectors for the app's spectrogram helper ``stft_mag_db`` (MS:197-212).

Container-only tool: imports the reference ``main_v2`` with GUI stubs (as
tools/gen_golden.py does) and writes inputs + the reference's outputs to
tests/golden/stft.npz (data only; float32 dB to keep the fixture small).

    python tools/gen_golden_stft.py
"""
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))
import numpy as np  # noqa: E402

from gen_golden import import_reference  # noqa: E402


def main():
    ms = import_reference()
    full = np.load(os.path.join(REPO, "tests", "golden", "render_full.npz"))
    out = {}
    # the mono mix the UI analyses (MS:1500): y.mean(axis=1) of a rendered buffer
    cases = {
        "c2": (full["C2_audio"].astype(np.float64)[:96000].mean(axis=1), 192000, 4096, 512, 3000),
        "defaults": (full["defaults_short_audio"].astype(np.float64).mean(axis=1), 48000, 2048, 256, 3000),
        "capped": (full["C1_audio"].astype(np.float64).mean(axis=1), 48000, 2048, 256, 40),
        "short": (full["C1_audio"].astype(np.float64)[:1500].mean(axis=1), 48000, 2048, 256, 3000),
        "odd": (full["C2odd_audio"].astype(np.float64)[:20001].mean(axis=1), 192000, 4096, 512, 3000),
    }
    for name, (x, sr, win, hop, mf) in cases.items():
        S = ms.stft_mag_db(x, sr, win=win, hop=hop, max_frames=mf)
        out[f"{name}_x"] = x
        out[f"{name}_S"] = S.astype(np.float32)
        out[f"{name}_cfg"] = np.array([sr, win, hop, mf], dtype=np.int64)
        print(name, x.shape, S.shape)
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "stft.npz"), **out)


if __name__ == "__main__":
    main()
