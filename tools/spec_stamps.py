#!/usr/bin/env python3
"""Per-phase time split of the spectral kernel (debug library with -DMSG_STAMPS).

    python audio-suite_amd/build.py --stamps
    MSGPU_LIB=audio-suite_amd/msgpu/libmsgpu_stamps.so python tools/spec_stamps.py [C3] [batch]
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
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0   # debug: 1 lowpass, 2 gathers, 4 transforms
irs = bench.load_irs()
packed = PackedBatch([msgpu.config_params(cfg, seed=1000 + b, irs=irs) for b in range(batch)])
eng = Engine(0)
out = eng.alloc_output(packed)
lib = L.lib()
# the compile-time-plan kernels (hot lengths) keep their own counters
fn = lib.msg_debug_stamps_ct if os.environ.get("MSGPU_SPEC_CT", "1") != "0" else lib.msg_debug_stamps
fn.argtypes = [C.POINTER(C.c_uint64), C.c_int]
buf = (C.c_uint64 * 16)()
lib.msg_debug_skip.argtypes = [C.c_int]
lib.msg_debug_skip(skip)
eng.render_packed(packed, out)
eng.torch.cuda.synchronize()
fn(buf, 16)                       # reset after warm-up
eng.render_packed(packed, out)
eng.torch.cuda.synchronize()
fn(buf, 16)
names = ["load", "twiddles", "tilt fwd+shape", "tilt inv+env", "chain fwd+ops", "chain inv",
         "-", "-", "-", "-", "store"]
tot = sum(buf[i] for i in range(11))
n_ev = sum(int(i.n_events) for i in eng.last_plan())
for i, nm in enumerate(names):
    print(f"{nm:14s} {buf[i] / max(1, n_ev) / 100.0:10.2f} us/event  {100.0 * buf[i] / max(1, tot):5.1f} %")
print("events", n_ev, "(wall_clock64 at 100 MHz), skip", skip)
