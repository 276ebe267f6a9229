"""Diagnostic: does a repeated render of the same batch on one engine give the
same audio?  Prints, per batch composition, which renders differ from the first."""
import os, sys, json
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "audio-suite_amd"))
import torch
import msgpu
from msgpu.engine import Engine
from msgpu.pack import PackedBatch

irs = dict(np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "irs.npz")))
info = json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "golden_info.json")))
params = [msgpu.config_params("C3", seed=1000, irs=irs, out_dur_s=0.3),
          msgpu.config_params("C2", seed=1001, irs=irs)]
for name in ("wavelet_mist", "02_friction_lattice", "chaotic_dustfield", "micro_carillon"):
    p = msgpu.merged(info["preset_params"][name]); p["out_dur_s"] = 0.5; p["_ir_audio"] = irs["tiny_room_ir"]
    params.append(p)
for proc in ("Clustered", "Hawkes", "Single"):
    params.append(msgpu.config_params("C2", seed=1002, irs=irs, event_process=proc, out_dur_s=0.5))
e = Engine(0)
def run(name, plist, reps=6, **over):
    pk = PackedBatch(plist)
    outs = []
    for r in range(reps):
        x = e.render_packed(pk); torch.cuda.synchronize(0); outs.append(x.cpu().numpy().copy())
    d = [float(np.abs(o - outs[0]).max()) for o in outs]
    print(f"{name:28s}", " ".join(f"{v:.2e}" for v in d), flush=True)
run("full batch", params)
run("wavelet alone", [params[2]])
run("p0,p1,wavelet", params[:3])
run("wavelet, no ER", [msgpu.merged(params[2], er_cloud_on=False)])
run("wavelet, no IR", [msgpu.merged(params[2], space_ir_on=False)])
run("wavelet, no FIR", [msgpu.merged(params[2], space_ir_on=False, er_cloud_on=False)])
run("p0,p1,wavelet no FIR", params[:2] + [msgpu.merged(params[2], space_ir_on=False, er_cloud_on=False)])
