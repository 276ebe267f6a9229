"""Diagnostic: device vs oracle error of one preset with output stages switched
off one at a time (ER, IR, stereo, saturation).  GPU box only."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "audio-suite_amd"), REPO]
import msgpu  # noqa: E402
from oracle import msound_oracle as O  # noqa: E402

irs = dict(np.load(os.path.join(REPO, "tests", "golden", "irs.npz")))
base = dict(base_sr=192000, out_dur_s=0.6826, gen_mode="Resonant strike", event_process="Poisson",
            space_ir_on=True, seed=21, er_cloud_on=True, space_ir_max_samps=8192, _ir_audio=irs["tiny_room_ir"])
variants = {
    "all": {}, "no_er": dict(er_cloud_on=False), "no_ir": dict(space_ir_on=False),
    "no_space": dict(er_cloud_on=False, space_ir_on=False), "no_stereo": dict(stereo_on=False),
    "no_stereo_space": dict(stereo_on=False, er_cloud_on=False, space_ir_on=False),
    "no_band": dict(bandlimit_on=False, stereo_on=False, er_cloud_on=False, space_ir_on=False),
    "drive0": dict(sat_drive=0.0),
}
for name, kw in variants.items():
    p = msgpu.merged(base, **kw)
    a, _ = msgpu.render(p)
    r, _ = O.render(p)
    d = np.abs(a.astype(np.float64) - r)
    i = np.unravel_index(np.argmax(d), d.shape)
    print(f"{name:16s} rms {np.sqrt(np.mean(d ** 2)):.3e} max {d.max():.3e} at {i} ref {r[i]:.6f}")
