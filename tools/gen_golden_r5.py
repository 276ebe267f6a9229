#!/usr/bin/env python3
"""Round-5 fixture: an output longer than 2^29 frames (VERDICT r04 missing #1).

One preset at 384 kHz for 1398.784 s = 2^29 + 2^18 frames, no ER / IR, a few
Poisson events at 2 / s (about 2 800 grains over the whole output, so they
land on both sides of frame 2^29), rendered by the reference itself
(microsound_0.2.1/main_v2.py's render, imported with tools/gen_golden.py's
stubs) in this container -- ~37 GB of host memory, a few
minutes.  The render is too large to commit; its summary is: rms, peak,
per-channel sums, the frames of every 2^20-th row, and the per-segment sums of
|L| and |R| over 512 equal segments (where the events are).  Round 5 made the
fixture with the NumPy restatement (oracle/msound_oracle.py); --check-oracle
renders that too and records whether its summary equals the reference's, field
for field (``oracle_equal``).

    python tools/gen_golden_r5.py [--check-oracle]   # writes tests/golden/long_2e29.json
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))
sys.path.insert(0, REPO)

N = (1 << 29) + (1 << 18)
SR = 384000


def params():
    import msgpu
    return msgpu.merged(seed=77, base_sr=SR, out_dur_s=N / SR, event_process="Poisson", grains_per_sec=2.0,
                        space_ir_on=False, er_cloud_on=False)


def summary(a):
    """Summary of an (N, 2) render, float64 accumulation (the GPU test computes the same)."""
    n = a.shape[0]
    seg = 512
    b = np.abs(a[: n - n % seg].astype(np.float64)).reshape(seg, -1, 2).sum(axis=1)
    return {"out_n": int(n), "rms": float(np.sqrt(np.mean(np.square(a, dtype=np.float64)))),
            "peak": float(np.max(np.abs(a))), "sum_l": float(a[:, 0].sum(dtype=np.float64)),
            "sum_r": float(a[:, 1].sum(dtype=np.float64)),
            "rows_every_2e20": a[:: 1 << 20].astype(np.float64).tolist(),
            "seg_abs_sums": b.tolist(), "seg": seg}


def main():
    import gc
    sys.dont_write_bytecode = True                 # nothing written under /root/reference
    sys.path.insert(0, os.path.join(REPO, "tools"))
    from gen_golden import import_reference
    ms = import_reference()
    t0 = time.time()
    a, meta = ms.render(params())
    assert a.shape == (N, 2), a.shape
    s = summary(a)
    s["source"] = "reference: microsound_0.2.1/main_v2.py render() (tools/gen_golden.py import_reference)"
    s["reference_seconds"] = round(time.time() - t0, 1)
    s["numpy"] = np.__version__
    del a, meta
    gc.collect()
    if "--check-oracle" in sys.argv:
        from oracle import msound_oracle as O
        t0 = time.time()
        b, _ = O.render(params())
        so = summary(b)
        del b
        gc.collect()
        keys = ("out_n", "rms", "peak", "sum_l", "sum_r", "rows_every_2e20", "seg_abs_sums")
        s["oracle_equal"] = {k: so[k] == s[k] for k in keys}
        s["oracle_seconds"] = round(time.time() - t0, 1)
    s["params"] = {"seed": 77, "base_sr": SR, "out_dur_s": N / SR, "event_process": "Poisson",
                   "grains_per_sec": 2.0, "space_ir_on": False, "er_cloud_on": False}
    s["active_segments"] = [i for i, v in enumerate(s["seg_abs_sums"]) if v[0] > 0]
    out = os.path.join(REPO, "tests", "golden", "long_2e29.json")
    with open(out, "w") as f:
        json.dump(s, f)
    print(out, s["rms"], s["peak"], len(s["active_segments"]), s["reference_seconds"], s.get("oracle_equal"))


if __name__ == "__main__":
    main()
