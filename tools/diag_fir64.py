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


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def meta_errors():
    """Relative RMS error of the device's micro_last / grain_last (float32 chain)
    against the oracle's, per case: the generator's and the spectral chain's share."""
    irs = dict(np.load(os.path.join(REPO, "tests", "golden", "irs.npz")))
    base = dict(gen_mode="Resonant strike", event_process="Single", _ir_audio=None, space_ir_on=False,
                er_cloud_on=False)
    for sr, unf, st in ((48000, 25.0, 1.0), (192000, 25.0, 1.0), (384000, 100.0, 2.0), (48000, 25.0, 2.0)):
        for mode in ("Resonant strike", "Gaussian click", "Noise burst"):
            p = msgpu.merged(base, gen_mode=mode, base_sr=sr, time_unfold=unf, partial_stretch=st, out_dur_s=0.05,
                             seed=7)
            a, m = msgpu.render(p)
            ra, rm = O.render(p)
            rel = lambda x, y: float(np.sqrt(np.mean((x - y) ** 2) / np.mean(y ** 2)))  # noqa: E731
            print(f"{sr} x{unf} st{st} {mode:16s} n={rm['micro_last'].size}: micro rel {rel(m['micro_last'], rm['micro_last']):.2e}"
                  f"  grain rel {rel(m['grain_last'], rm['grain_last']):.2e}", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "meta":
    meta_errors()


def variants():
    """R48 (48 kHz ER + IR, 0.7 s) with one factor changed at a time, float64 FIR forced."""
    irs = dict(np.load(os.path.join(REPO, "tests", "golden", "irs.npz")))
    base = dict(gen_mode="Resonant strike", event_process="Poisson", _ir_audio=irs["tiny_room_ir"], base_sr=48000,
                out_dur_s=0.7, space_ir_on=True, seed=22, er_cloud_on=True, space_ir_max_samps=8192, stereo_width=0.3)
    vs = {"base": {}, "gauss": dict(gen_mode="Gaussian click"), "noise": dict(gen_mode="Noise burst"),
          "flat_env": dict(env_a=0.0, env_d=0.0, env_s=1.0, env_r=0.0), "no_band": dict(bandlimit_on=False),
          "no_stereo": dict(stereo_on=False), "drive0": dict(sat_drive=0.0), "no_er": dict(er_cloud_on=False),
          "unfold1": dict(time_unfold=1.0)}
    os.environ["MSGPU_FIR64"] = "2"
    from msgpu.engine import Engine
    from msgpu.pack import PackedBatch
    import torch
    eng = Engine(0)
    os.environ.pop("MSGPU_FIR64", None)
    for name, kw in vs.items():
        p = msgpu.merged(base, **kw)
        ref, _ = O.render(p)
        o = eng.render_packed(PackedBatch([p]))
        torch.cuda.synchronize(0)
        print(f"R48 {name:10s}: rms err {rms(o.cpu().numpy(), ref):.3e}", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "variants":
    variants()


def gen_detail():
    """Where the resonant strike's float32 error sits within one grain."""
    for sr, unf in ((48000, 25.0), (384000, 100.0)):
        p = msgpu.merged(gen_mode="Resonant strike", event_process="Single", base_sr=sr, time_unfold=unf,
                         out_dur_s=0.05, seed=7, er_cloud_on=False, space_ir_on=False)
        _, m = msgpu.render(p)
        _, rm = O.render(p)
        g, r = np.asarray(m["micro_last"], np.float64), rm["micro_last"]
        n = r.size
        e = g - r
        np.savez(os.path.join(REPO, "gpurun_out", f"gen_{sr}.npz"), g=g, r=r)
        rr = np.sqrt(np.mean(r ** 2))
        print(f"{sr}: n {n} rel {np.sqrt(np.mean(e ** 2)) / rr:.2e}; max |e| {np.abs(e).max():.2e} at {np.abs(e).argmax()}")
        for a, b in ((0, 64), (64, 512), (512, n // 4), (n // 4, n // 2), (n // 2, n - 64), (n - 64, n)):
            print(f"   [{a},{b}) rms e {np.sqrt(np.mean(e[a:b] ** 2)):.2e} rms r {np.sqrt(np.mean(r[a:b] ** 2)):.2e}"
                  f" corr(e, r) {np.corrcoef(e[a:b], r[a:b])[0, 1]:.2f}")
        print("   e[:8]", np.array2string(e[:8], precision=2), "r[:8]", np.array2string(r[:8], precision=3))
        rat = e[64:512] / np.where(np.abs(r[64:512]) > 1e-3, r[64:512], np.nan)
        print(f"   e/r [64,512): median {np.nanmedian(rat):.2e} std {np.nanstd(rat):.2e}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "gen":
    gen_detail()
