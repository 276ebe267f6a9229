import os, sys, time, json
sys.path.insert(0, '/root/repo/audio-suite_amd'); sys.path.insert(0, '/root/repo')
import numpy as np, torch
import msgpu
from msgpu.engine import Engine
from msgpu.pack import PackedBatch
z = np.load('/root/repo/tests/golden/irs.npz'); irs = {k: z[k] for k in z.files}
B = 1024
params = [msgpu.config_params("C3", seed=1000 + b, irs=irs) for b in range(B)]
for S in (1, 2, 4):
    subs = [PackedBatch(params[i * B // S:(i + 1) * B // S]) for i in range(S)]
    engs = [Engine(0) for _ in range(S)]
    outs = [e.alloc_output(p) for e, p in zip(engs, subs)]
    strs = [torch.cuda.Stream() for _ in range(S)]
    for _ in range(3):
        for e, p, o, s in zip(engs, subs, outs, strs): e.render_packed(p, o, s)
    torch.cuda.synchronize()
    K = 10
    t0 = time.perf_counter()
    for _ in range(K):
        for e, p, o, s in zip(engs, subs, outs, strs): e.render_packed(p, o, s)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K
    print(f"streams={S}: {dt*1e3:.3f} ms/step  {B*384000/dt/1e6:.0f} Msamples/s", flush=True)
    for e in engs: e.close()
    del outs
    torch.cuda.empty_cache()
