#!/usr/bin/env python3
"""Rehearse the multi-GPU library path on a one-GPU box (GPU box only).

msgpu.DevicePool([0] * W, share_devices=True) starts W spawn workers that all
render on device 0, before this process touches the GPU; a mixed batch (C2,
C3, H48 and default presets, so the cost cut is uneven) goes through
pool.render_batch, then the same batch renders in this process with
msgpu.render_batch(device=0) and the two are compared preset by preset.

    python tools/multi_rehearsal.py [W]     # prints one JSON line
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))


def main():
    w = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    import msgpu
    z = np.load(os.path.join(REPO, "tests", "golden", "irs.npz"))
    irs = {k: z[k] for k in z.files}
    params = []
    for i in range(24):
        cfg = ("C2", "C3", "H48", "C3")[i % 4]
        params.append(msgpu.config_params(cfg, seed=2000 + i, irs=irs))
    params.append(msgpu.merged({"seed": 7, "out_dur_s": 0.5}))
    pool = msgpu.DevicePool([0] * w, share_devices=True)     # before any GPU call here
    t0 = time.perf_counter()
    outs = pool.render_batch(params)
    t_pool = time.perf_counter() - t0
    split, workers = pool.last_split, pool.workers
    pool.close()
    t0 = time.perf_counter()
    ref = msgpu.render_batch(params, device=0)
    t_one = time.perf_counter() - t0
    diffs, exact = [], 0
    for a, b in zip(outs, ref):
        assert a.shape == b.shape and a.dtype == np.float32, (a.shape, b.shape)
        d = float(np.sqrt(np.mean((a.astype(np.float64) - b) ** 2)))
        diffs.append(d)
        exact += int(np.array_equal(a, b))
    ok = len(outs) == len(params) and max(diffs) <= 1e-6
    print(json.dumps({"workers": workers, "split": split, "presets": len(params), "bit_exact": exact,
                      "max_rms_diff": max(diffs), "ok": ok, "pool_s": round(t_pool, 3),
                      "in_process_s": round(t_one, 3)}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
