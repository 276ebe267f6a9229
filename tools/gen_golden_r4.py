#!/usr/bin/env python3
"""Round-4 golden vectors, from the reference ``render`` itself.

Container-only tool (imports microsound_0.2.1/main_v2.py with the GUI modules
stubbed, exactly as tools/gen_golden.py does).  Writes DATA fixtures
``tests/golden/render_r4.npz`` + ``tests/golden/golden_r4.json``:

* breakpoint lanes of 40 and 200 points on all four lanes (density, unfold,
  cutoff, stretch; MS:452-482, 602-605, 634-637) -- the lanes are free-text
  fields in the UI (MS:1070-1073), so any count is reachable; unsorted input with
  repeated times, so parse_breakpoints' stable sort (MS:466) matters;
* counts beyond the UI's spin boxes, reachable through preset JSON: 300
  resonator modes (MS:369-384; UI max 128, MS:1079), 300 wavelet atoms
  (MS:317-331; UI max 64, MS:976), 300 waveguide lines (MS:386-402; UI max 32,
  MS:1089), and partial locking of 300 peaks (MS:130-148; UI max 200, MS:995);
* an ER + IR filter longer than the output (192 kHz, er_max_ms 150, 0.17 s:
  28 800 + 8192 taps over 32 640 frames).

Every case stores the whole (out_n, 2) buffer as float32 plus its summary.

    python tools/gen_golden_r4.py
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))

from gen_golden import import_reference, load_irs, summary  # noqa: E402
from msgpu.params import merged  # noqa: E402

OUT = os.path.join(REPO, "tests", "golden")


def lane(npts, seed, t_max, lo, hi):
    """npts 't:v' points, shuffled, one time repeated (stable sort keeps input order)."""
    rng = np.random.default_rng(seed)
    t = np.round(rng.uniform(0.0, t_max, npts), 4)
    t[npts // 3] = t[npts // 2]
    v = np.round(rng.uniform(lo, hi, npts), 3)
    return ", ".join(f"{t[i]}:{v[i]}" for i in rng.permutation(npts))


def cases(irs):
    tiny = irs["tiny_room_ir"]
    out = {}
    for npts in (40, 200):
        out[f"LANES{npts}"] = merged(
            gen_mode="Resonant strike", event_process="Poisson", grains_per_sec=60.0, base_sr=48000,
            out_dur_s=0.6, seed=400 + npts, time_unfold=10.0, partial_stretch=1.5, space_ir_on=True,
            space_ir_max_samps=2048, _ir_audio=tiny,
            bp_density=lane(npts, 1 + npts, 0.7, 4.0, 60.0), bp_unfold=lane(npts, 2 + npts, 0.7, 2.0, 24.0),
            bp_cutoff=lane(npts, 3 + npts, 0.7, 1500.0, 20000.0), bp_stretch=lane(npts, 4 + npts, 0.7, 0.5, 3.0))
    base = dict(event_process="Poisson", grains_per_sec=12.0, base_sr=48000, out_dur_s=0.3, time_unfold=4.0,
                _ir_audio=None)
    out["RES300"] = merged(base, gen_mode="Gaussian click", seed=501, res_bank_on=True, res_modes=300,
                           res_fmin=80.0, res_fmax=20000.0, res_decay_ms=30.0)
    out["WAV300"] = merged(base, gen_mode="Wavelet atoms", seed=502, wav_count=300, wav_spread=1.2)
    out["WG300"] = merged(base, gen_mode="Noise burst", seed=503, wg_on=True, wg_lines=300, wg_max_ms=3.0,
                          wg_fb=0.5, grains_per_sec=8.0)
    out["PL300"] = merged(base, gen_mode="Noise burst", seed=504, partial_lock_on=True, pl_top_n=300,
                          pl_neigh=3, partial_stretch=1.3, time_unfold=16.0)
    out["CLIP192"] = merged(gen_mode="Resonant strike", event_process="Poisson", base_sr=192000, out_dur_s=0.17,
                            seed=505, er_cloud_on=True, er_max_ms=150.0, er_taps=600, space_ir_on=True,
                            space_ir_max_samps=8192, _ir_audio=tiny)
    return out


def main():
    ms = import_reference()
    irs = load_irs()
    arrays, info = {}, {"summaries": {}, "params": {}, "timings_s": {}, "numpy": np.__version__,
                        "generator": "tools/gen_golden_r4.py"}
    for name, p in cases(irs).items():
        t0 = time.time()
        audio, meta = ms.render(p)
        dt = time.time() - t0
        info["summaries"][name] = summary(audio)
        info["summaries"][name]["design_sr_base"] = int(meta["design_sr_base"])
        info["timings_s"][name] = dt
        info["params"][name] = {k: v for k, v in p.items() if not k.startswith("_")}
        if p.get("_ir_audio") is not None:
            info["params"][name]["_ir"] = "tiny_room_ir"
        arrays[f"{name}_audio"] = audio.astype(np.float32)
        print(f"{name}: {audio.shape} {dt:.1f}s", flush=True)
    np.savez_compressed(os.path.join(OUT, "render_r4.npz"), **arrays)
    with open(os.path.join(OUT, "golden_r4.json"), "w") as fh:
        json.dump(info, fh, indent=1)


if __name__ == "__main__":
    main()
