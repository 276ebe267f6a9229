#!/usr/bin/env python3
"""GPU diagnostic: where the error of saturated ER + IR renders comes from.

For each case: the device render with the float32 FIR (MSGPU_FIR64=0) and the
float64 FIR forced (=2) against the oracle, and the standalone device FIR
(msg_fir, float32) applied to the oracle's exact mono with the exact h, run
through the oracle's output stage -- the float32 FIR's share alone.

    python tools/diag_fir64.py   (on the GPU box)
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "audio-suite_amd"), REPO, os.path.join(REPO, "tools")):
    sys.path.insert(0, p)

import fir_error_model as M  # noqa: E402
import msgpu  # noqa: E402
from oracle import msound_oracle as O  # noqa: E402


def rms(a, b):
    return float(np.sqrt(np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)))


def main():
    import torch
    from msgpu.engine import Engine
    from msgpu.pack import PackedBatch
    irs = dict(np.load(os.path.join(REPO, "tests", "golden", "irs.npz")))
    base = dict(gen_mode="Resonant strike", event_process="Poisson", _ir_audio=irs["tiny_room_ir"])
    cases = {
        "R48": msgpu.merged(base, base_sr=48000, out_dur_s=0.7, space_ir_on=True, seed=22, er_cloud_on=True,
                            space_ir_max_samps=8192, stereo_width=0.3),
        "R48b": msgpu.merged(base, base_sr=48000, out_dur_s=0.3, space_ir_on=True, seed=21, er_cloud_on=True,
                             space_ir_max_samps=8192),
        "ERIR192def": msgpu.merged(base, base_sr=192000, out_dur_s=0.6826, space_ir_on=True, seed=21,
                                   er_cloud_on=True, space_ir_max_samps=8192),
    }
    for name, p in cases.items():
        ref, _ = O.render(p)
        line = [name]
        for m in ("0", "2"):
            os.environ["MSGPU_FIR64"] = m
            try:
                eng = Engine(0)
            finally:
                os.environ.pop("MSGPU_FIR64", None)
            pk = PackedBatch([p])
            o = eng.render_packed(pk)
            torch.cuda.synchronize(0)
            line.append(f"render FIR64={m}: {rms(o.cpu().numpy(), ref):.3e}")
        x, sr = M.mono_of(p)
        h = M.space_h(p, x.size, sr)
        y_exact = np.convolve(x, h)[:x.size]
        xd = torch.from_numpy(x.astype(np.float32)).to("cuda:0")
        yd, shape = eng.fir(xd, h[:x.size])
        torch.cuda.synchronize(0)
        y32 = yd.cpu().numpy().astype(np.float64)
        line.append(f"msg_fir(exact x) {shape}: {rms(M.tail(p, y32, sr), ref):.3e}")
        line.append(f"y rel err {np.sqrt(np.mean((y32 - y_exact) ** 2) / np.mean(y_exact ** 2)):.2e}")
        line.append(f"exact-y oracle tail: {rms(M.tail(p, y_exact, sr), ref):.1e}")
        print(" | ".join(line), flush=True)


if __name__ == "__main__":
    main()
