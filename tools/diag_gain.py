"""Diagnostic: split a device render's error vs the oracle into a global gain
part (peak normalisation, MS:781) and the rest.  GPU box only."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "audio-suite_amd"), REPO]
import msgpu  # noqa: E402
from oracle import msound_oracle as O  # noqa: E402

irs = dict(np.load(os.path.join(REPO, "tests", "golden", "irs.npz")))
cases = {
    "fir192q2": msgpu.merged(base_sr=192000, out_dur_s=0.6826, gen_mode="Resonant strike", event_process="Poisson",
                             space_ir_on=True, seed=21, er_cloud_on=True, space_ir_max_samps=8192,
                             _ir_audio=irs["tiny_room_ir"]),
    "erir192": msgpu.merged(base_sr=192000, out_dur_s=0.3, gen_mode="Resonant strike", event_process="Poisson",
                            seed=1000, er_cloud_on=True, er_max_ms=150.0, space_ir_on=True, space_ir_max_samps=8192,
                            _ir_audio=irs["tiny_room_ir"]),
    "C3": msgpu.config_params("C3", seed=1000, irs=irs),
}
for name, p in cases.items():
    a, _ = msgpu.render(p)
    r, _ = O.render(p)
    a = a.astype(np.float64)
    e = np.sqrt(np.mean((a - r) ** 2))
    g = float(np.sum(a * r) / np.sum(a * a))
    e2 = np.sqrt(np.mean((g * a - r) ** 2))
    i = np.unravel_index(np.argmax(np.abs(r)), r.shape)
    print(f"{name}: rms {e:.3e}  gain-fit {g - 1:+.3e} residual {e2:.3e}  max|d| {np.max(np.abs(a - r)):.3e}"
          f"  peak frame {i} dev {a[i]:.9f} ref {r[i]:.9f}")
