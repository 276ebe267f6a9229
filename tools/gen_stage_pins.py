#!/usr/bin/env python3
"""Golden inputs of the two ill-conditioned stages, from the reference itself.

Container-only tool (imports microsound_0.2.1/main_v2.py with the GUI modules
stubbed, as tools/gen_golden.py does).  For the seven presets whose full render
the tests hold to the reference's own rounding spread (render_spread.json), it
renders the preset as tests/golden/render_full.npz does (0.5 s, tiny-room IR,
the golden image) with the reference's ``cepstral_warp`` (MS:150-163) and
``SpectralImprint.apply`` (MS:565-581) wrapped, and records the grain each call
receives for the render's LAST event -- the float64 chain's state just before
the step whose result depends on float64 rounding (log(|X| + 1e-12), angle(X)).
Writes the DATA fixture tests/golden/stage_pins.npz; tests/test_gpu_stage_pins.py
holds the device's float64 chain to <= 1e-9 (relative RMS) at those points.

    python tools/gen_stage_pins.py
"""
from __future__ import annotations

import json
import os
import sys

sys.dont_write_bytecode = True

import numpy as np  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))

from gen_golden import REF_DIR, import_reference, load_irs  # noqa: E402
from msgpu.params import merged  # noqa: E402

PRESETS = ["ghost_formants", "03_wavelet_ice_bloom", "wavelet_mist", "closed_curve_air",
           "drifting_mode_fragments", "corona_glass_fog", "soft_ellipse_memory"]


def main():
    ms = import_reference()
    irs = load_irs()
    img = (np.add.outer(np.arange(48), np.arange(64)) * 7 % 256).astype(np.uint8)   # as gen_golden.py
    rec = {}
    cep0, imp0 = ms.cepstral_warp, ms.SpectralImprint.apply

    def cep(x, *a, **k):
        rec["cep"] = np.array(x, dtype=np.float64, copy=True)
        return cep0(x, *a, **k)

    def imp(self, grain, *a, **k):
        rec["imp"] = np.array(grain, dtype=np.float64, copy=True)
        return imp0(self, grain, *a, **k)

    ms.cepstral_warp = cep
    ms.SpectralImprint.apply = imp
    out, info = {}, {}
    for name in PRESETS:
        with open(os.path.join(REF_DIR, "presets", f"{name}.json"), encoding="utf-8") as fh:
            p = merged(json.load(fh))
        p["out_dur_s"] = 0.5
        p["_ir_audio"] = irs["tiny_room_ir"]
        p["_img_gray"] = img
        rec.clear()
        ms.render(p)
        info[name] = sorted(rec)
        for k, v in rec.items():
            out[f"{name}_{k}"] = v
        print(name, {k: v.shape for k, v in rec.items()})
    ms.cepstral_warp, ms.SpectralImprint.apply = cep0, imp0
    out["info"] = np.array(json.dumps({"numpy": np.__version__, "stages": info,
                                       "generator": "tools/gen_stage_pins.py"}))
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "stage_pins.npz"), **out)


if __name__ == "__main__":
    main()
