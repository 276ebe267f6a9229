#!/usr/bin/env python3
"""Standalone FIR benchmark (SURVEY §8 config remarks, §8(d)): y = np.convolve(x, h)[:n]
with 16 384- and 65 536-tap synthetic IRs over C3-length signals (n = 384 000), one
batch of S signals per call through msg_fir (k_ir_spec + k_fir2).

    python tools/fir_bench.py [--batch 1024] [--steps 10] [--taps 16384,65536] [--cpu]

Prints one JSON line per tap count: Msamples/s (output samples), ms per call, the
k_fir2 kernel time from HIP events around the launch sequence on the call's
stream, and algorithmic bytes 8 n + 4 M per signal against 8 TB/s.
With --cpu, also times np.convolve (the reference arithmetic, 1 core) on one signal.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--n", type=int, default=384000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--taps", default="16384,65536,262144")
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args()
    import torch
    from msgpu.engine import Engine
    from oracle import msound_oracle as O

    eng = Engine(0)
    dev = torch.device("cuda:0")
    S, n = a.batch, a.n
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    x = torch.randn((S, n), generator=g, device=dev, dtype=torch.float32)
    y = torch.empty_like(x)
    stream = torch.cuda.current_stream(dev)
    for M in (int(t) for t in a.taps.split(",")):
        h = O.synthetic_fir_taps(M)
        for _ in range(a.warmup):
            eng.fir(x, h, out=y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(a.steps):
            _, shape = eng.fir(x, h, out=y)
        e1.record(stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / a.steps
        dev_ms = e0.elapsed_time(e1) / a.steps
        alg = S * (8.0 * n + 4.0 * M)
        line = {"bench": "standalone_fir", "taps": M, "signals": S, "n": n,
                "fir_shape": {"N": shape[0], "P": shape[1], "Q": shape[2]},
                "ms_per_call": round(wall * 1e3, 4), "device_ms_per_call": round(dev_ms, 4),
                "msamples_per_s": round(S * n / wall / 1e6, 1),
                "algorithmic_bytes": alg, "achieved_GBs": round(alg / (dev_ms * 1e-3) / 1e9, 1),
                "peak_GBs": 8000.0, "frac": round(alg / (dev_ms * 1e-3) / 8e12, 4)}
        if a.cpu:
            xs = x[0].cpu().numpy().astype(np.float64)
            t0 = time.perf_counter()
            O.fir_causal(xs, h)
            dt = time.perf_counter() - t0
            line["cpu_baseline"] = {"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": 1,
                                    "kind": "port", "sample": f"np.convolve of one {n}-sample signal"}
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
