#!/usr/bin/env python3
"""Bit-for-bit A/B of two builds of libmsgpu on a mixed batch (GPU box).

A change that only moves data differently (load widths, store order, launch
shapes) must leave every output bit as it was.  Each library renders the same
batch in its own process (MSGPU_LIB selects the build; the ctypes binding loads
one library per process); the outputs are compared here.

    python tools/bits_ab.py audio-suite_amd/msgpu/libmsgpu_base.so [other.so]
    python tools/bits_ab.py 'lib.so,MSGPU_X=0' 'lib.so,MSGPU_X=1'

The second library defaults to the product build.  A side may add KEY=VALUE
settings after commas (the same library under two settings).  Prints one JSON
line and exits non-zero when any preset differs.
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def batch():
    sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))
    import msgpu
    z = np.load(os.path.join(REPO, "tests", "golden", "irs.npz"))
    irs = {k: z[k] for k in z.files}
    base = dict(gen_mode="Resonant strike", event_process="Poisson", _ir_audio=irs["tiny_room_ir"])
    ps = [msgpu.config_params("C3", seed=1000 + s, irs=irs) for s in range(3)]
    ps += [msgpu.config_params("C4", seed=1000, irs=irs), msgpu.config_params("H48", seed=1000, irs=irs),
           msgpu.config_params("C2", seed=1000, irs=irs),
           msgpu.config_params("C5", seed=1000, irs=irs, out_dur_s=30.0),
           msgpu.merged(out_dur_s=0.2000208, seed=6, base_sr=48000),                          # odd length
           msgpu.merged(out_dur_s=0.3, seed=7, stereo_on=False),                              # no rotation
           msgpu.merged(out_dur_s=0.3, seed=8, sat_drive=0.0),                                # no tanh
           msgpu.merged(base, base_sr=48000, out_dur_s=0.3, space_ir_on=True, seed=22, er_cloud_on=True,
                        space_ir_max_samps=8192, stereo_width=0.3),                            # float64 FIR
           msgpu.merged(out_dur_s=0.0013, seed=9, env_a=0.0, env_r=0.5),                     # under one tile
           msgpu.merged(out_dur_s=1.5, seed=10, stereo_width=1.0, base_sr=44100)]
    for i in range(5):                                                                         # odd offsets
        ps.append(msgpu.merged(out_dur_s=0.1 + 0.0000227 * i, seed=40 + i, base_sr=44100))
    return ps


def child(out):
    sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))
    import msgpu
    import torch
    from msgpu.engine import Engine
    from msgpu.pack import PackedBatch
    ps = batch()
    eng = Engine(0)
    packed = PackedBatch(ps)
    o = eng.render_packed(packed)
    torch.cuda.synchronize(0)
    np.savez(out, out=o.cpu().numpy(), offsets=np.asarray(packed.offsets), out_n=np.asarray(packed.out_n),
             lib=np.array(msgpu._lib.LIB_PATH))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        return child(sys.argv[2])
    sides = [sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "audio-suite_amd", "msgpu",
                                                                           "libmsgpu.so")]
    libs, envs = [], []
    for side in sides:
        lib, *kv = side.split(",")
        libs.append(os.path.abspath(lib))
        envs.append(dict(x.split("=", 1) for x in kv))
    tmp = tempfile.mkdtemp()
    res = []
    for k, lib in enumerate(libs):
        f = os.path.join(tmp, f"{k}.npz")
        subprocess.check_call([sys.executable, os.path.abspath(__file__), "--child", f],
                              env=dict(os.environ, MSGPU_LIB=lib, **envs[k]))
        res.append(np.load(f))
    a, b = res[0]["out"], res[1]["out"]
    diff = []
    for i, (o, n) in enumerate(zip(res[0]["offsets"], res[0]["out_n"])):
        if not np.array_equal(a[o:o + n], b[o:o + n]):
            diff.append(i)
    print(json.dumps({"libs": libs, "envs": envs, "presets": len(res[0]["out_n"]), "frames": int(res[0]["out_n"].sum()),
                      "differing_presets": diff, "identical": not diff}), flush=True)
    sys.exit(0 if not diff else 1)


if __name__ == "__main__":
    main()
