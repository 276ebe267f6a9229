#!/usr/bin/env python3
"""Per-phase time split of k_spec3 (an experiment library with -DMSG_STAMPS in k_spec3.hip).

    MSGPU_EXP_DEFS=-DMSG_STAMPS python audio-suite_amd/build.py --exp-tu k_spec3.hip --out libmsgpu_s3stamps.so
    MSGPU_LIB=audio-suite_amd/msgpu/libmsgpu_s3stamps.so python tools/spec3_stamps.py [C3] [batch]
"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import msgpu  # noqa: E402
from msgpu import _lib as L  # noqa: E402
from msgpu.engine import Engine  # noqa: E402
from msgpu.pack import PackedBatch  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 256
irs = bench.load_irs()
packed = PackedBatch([msgpu.config_params(cfg, seed=1000 + b, irs=irs) for b in range(batch)])
eng = Engine(0)
out = eng.alloc_output(packed)
fn = L.lib().msg_debug_stamps_s3
fn.argtypes = [C.POINTER(C.c_uint64), C.c_int]
buf = (C.c_uint64 * 16)()
eng.render_packed(packed, out)
eng.torch.cuda.synchronize()
fn(buf, 16)
eng.render_packed(packed, out)
eng.torch.cuda.synchronize()
fn(buf, 16)
# stamp 7 (wide band only) closes the Y gather; stamp 4 then holds inverse pass 1 alone
names = ["setup+F pass1 (HBM)", "F pass2", "F pass3+band Z", "split+mask", "I pass1 (gather)", "I pass2",
         "I pass3 (HBM)", "wide: Y gather"]
order = [0, 1, 2, 3, 7, 4, 5, 6]
tot = sum(buf[i] for i in range(8))
n_ev = sum(int(i.n_events) for i in eng.last_plan())
for i in order:
    nm = names[i]
    print(f"{nm:22s} {buf[i] / max(1, n_ev) / 100.0:10.2f} us/event  {100.0 * buf[i] / max(1, tot):5.1f} %")
print("events", n_ev, "(wall_clock64 at 100 MHz)")
