"""Diagnostic: per-preset differences between two renders of one batch
(host plan twice, device plan once).  Run on the GPU box from the repo root."""
import os, sys, json
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "audio-suite_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import torch
import msgpu
from msgpu.engine import Engine
from msgpu.pack import PackedBatch

irs = dict(np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "irs.npz")))
info = json.load(open(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "golden_info.json")))
irs_named = {k: v for k, v in irs.items()}
params = [msgpu.config_params("C3", seed=1000, irs=irs_named, out_dur_s=0.3),
          msgpu.config_params("C2", seed=1001, irs=irs_named)]
for name in ("wavelet_mist", "02_friction_lattice", "chaotic_dustfield", "micro_carillon"):
    p = msgpu.merged(info["preset_params"][name]); p["out_dur_s"] = 0.5; p["_ir_audio"] = irs_named["tiny_room_ir"]
    params.append(p)
for proc in ("Clustered", "Hawkes", "Single"):
    params.append(msgpu.config_params("C2", seed=1002, irs=irs_named, event_process=proc, out_dur_s=0.5))
packed = PackedBatch(params)
e1 = Engine(0)
a = e1.render_packed(packed); torch.cuda.synchronize(0); a = a.cpu().numpy().copy()
b = e1.render_packed(packed); torch.cuda.synchronize(0); b = b.cpu().numpy().copy()
os.environ["MSGPU_DEVICE_PLAN"] = "1"
e2 = Engine(0)
c = e2.render_packed(packed); torch.cuda.synchronize(0); c = c.cpu().numpy().copy()
print("host-host max", float(np.max(np.abs(a - b))), "host-dev max", float(np.max(np.abs(a - c))))
os.environ.pop("MSGPU_DEVICE_PLAN")
for rep in range(4):   # concurrent: both engines in flight before the synchronize (as the test)
    x = e1.render_packed(packed); y = e2.render_packed(packed); torch.cuda.synchronize(0)
    x, y = x.cpu().numpy(), y.cpu().numpy()
    dd = np.abs(x - y).max(axis=1); bad = np.nonzero(dd > 1e-6)[0]
    print("concurrent rep", rep, "max", float(dd.max()), "bad frames", bad.size, bad[:5], "vs a", float(np.abs(x - a).max()), float(np.abs(y - a).max()))
for rep in range(2):   # same engine twice in flight
    x = e1.render_packed(packed); y = e1.render_packed(packed); torch.cuda.synchronize(0)
    print("same-engine rep", rep, float(np.abs(x.cpu().numpy() - a).max()), float(np.abs(y.cpu().numpy() - a).max()))
for k, p in enumerate(params):
    pk = PackedBatch([p])
    x = e1.render_packed(pk); y = e2.render_packed(pk); z = e1.render_packed(pk); torch.cuda.synchronize(0)
    x, y, z = x.cpu().numpy(), y.cpu().numpy(), z.cpu().numpy()
    dd = np.abs(x - y).max(axis=1)
    print(k, p.get("gen_mode"), p.get("event_process"), "host-dev", float(dd.max()), "host-host", float(np.abs(x - z).max()),
          "first bad frame", int(np.argmax(dd > 1e-6)) if (dd > 1e-6).any() else None, "n", x.shape[0])
