#!/usr/bin/env python3
"""Rehearse the multi-GPU library path on a one-GPU box (GPU box only).

msgpu.DevicePool([0] * W, share_devices=True) starts W spawn workers that all
render on device 0, before this process touches the GPU; a mixed batch (C2,
C3, H48 and default presets, so the cost cut is uneven) goes through
pool.render_batch, then the same batch renders in this process with
msgpu.render_batch(device=0) and the two are compared preset by preset.

    python tools/multi_rehearsal.py [W]     # prints one JSON line

``stats W N``: N C5 presets (seeds 1000..) through pool.render_batch(...,
results="stats") -- the C5-scale mode that never brings the outputs (67 MB per
preset) to the host: each render is reduced on the device (msg_digest) and 48
bytes per preset cross PCIe.  The same pool first renders the batch with
results="device" (renders kept in HBM, then released), so stats_overhead_s is
what the summaries cost beyond the render itself.  Records the parent's and the
workers' peak RSS, checks preset 0 against the reference's C5 summary and the
first presets' summaries against the same presets rendered in this process
afterwards.
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))


def stats_main(w, n):
    import resource
    import msgpu
    z = np.load(os.path.join(REPO, "tests", "golden", "irs.npz"))
    irs = {k: z[k] for k in z.files}
    with open(os.path.join(REPO, "tests", "golden", "golden_info.json")) as f:
        golden = json.load(f)["summaries"]
    params = [msgpu.config_params("C5", seed=1000 + i, irs=irs) for i in range(n)]
    rss0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    pool = msgpu.DevicePool([0] * w, share_devices=True)     # before any GPU call here
    pool.render_batch(params[:w], results="stats")             # warm the workers (plans, buffers)
    t0 = time.perf_counter()
    hs = pool.render_batch(params, results="device")
    t_dev = time.perf_counter() - t0
    pool.release(hs)
    t0 = time.perf_counter()
    stats = pool.render_batch(params, results="stats")
    t_pool = time.perf_counter() - t0
    split = pool.last_split
    pool.close()
    rss_parent = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    rss_workers = resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss
    ref = golden.get("C5_1000")
    d0 = {"rms": abs(stats[0]["rms"] - ref["rms"]), "sum_l": abs(stats[0]["sum_l"] - ref["sum_l"]) / stats[0]["out_n"],
          "sum_r": abs(stats[0]["sum_r"] - ref["sum_r"]) / stats[0]["out_n"]} if ref else None
    k = min(4, n)
    again = msgpu.render_batch(params[:k], device=0, results="stats")
    same = all(a == b for a, b in zip(stats[:k], again))
    out_bytes = 8 * sum(s["out_n"] for s in stats)
    ok = len(stats) == n and same and (d0 is None or max(d0.values()) <= 1e-5)
    print(json.dumps({"mode": "stats", "workers": w, "presets": n, "split": split, "pool_s": round(t_pool, 2),
                      "device_mode_s": round(t_dev, 2), "stats_overhead_s": round(t_pool - t_dev, 2),
                      "output_bytes_in_hbm": out_bytes, "bytes_copied_to_host": 48 * n,
                      "parent_maxrss_mb": round(rss_parent / 1024, 1),
                      "parent_maxrss_before_mb": round(rss0 / 1024, 1),
                      "workers_maxrss_mb": round(rss_workers / 1024, 1),
                      "preset0_vs_reference": d0, "first_presets_equal_in_process": same,
                      "stats0": stats[0], "ok": ok}), flush=True)
    sys.exit(0 if ok else 1)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "stats":
        return stats_main(int(sys.argv[2]) if len(sys.argv) > 2 else 2, int(sys.argv[3]) if len(sys.argv) > 3 else 1024)
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
