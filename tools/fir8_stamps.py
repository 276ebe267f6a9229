#!/usr/bin/env python3
"""Per-phase time split of k_fir8 (an experiment library with -DMSG_STAMPS in k_fir.hip).

    MSGPU_EXP_DEFS=-DMSG_STAMPS python audio-suite_amd/build.py --exp-tu k_fir.hip --out libmsgpu_firstamps.so
    MSGPU_LIB=audio-suite_amd/msgpu/libmsgpu_firstamps.so python tools/fir8_stamps.py [C3] [batch]

Each phase ends at a barrier, so the split is of the block's wall time; the sum
over phases divided by the number of blocks is the mean block duration.
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
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
irs = bench.load_irs()
packed = PackedBatch([msgpu.config_params(cfg, seed=1000 + b, irs=irs) for b in range(batch)])
eng = Engine(0)
out = eng.alloc_output(packed)
fn = L.lib().msg_debug_stamps_fir
fn.argtypes = [C.POINTER(C.c_uint64), C.c_int]
buf = (C.c_uint64 * 16)()
eng.render_packed(packed, out)
eng.torch.cuda.synchronize()
fn(buf, 16)
eng.render_packed(packed, out)
eng.torch.cuda.synchronize()
fn(buf, 16)
names = ["segment + tables load, DIF split", "forward even half", "even MAC (He loads) + pre-step",
         "inverse even half", "forward odd half", "odd MAC (Ho loads) + pre-step", "inverse odd half",
         "DIT join + stores"]
tot = sum(buf[i] for i in range(8))
blocks = 0
for i, inf in enumerate(eng.last_plan()):
    n = int(inf.out_n)
    blocks += -(-n // 40064)          # C3/C4: B = 65536 - 25473 + 1
for i, nm in enumerate(names):
    print(f"{nm:34s} {buf[i] / max(1, blocks) / 100.0:9.2f} us/block  {100.0 * buf[i] / max(1, tot):5.1f} %")
print(f"{'total':34s} {tot / max(1, blocks) / 100.0:9.2f} us/block  ({blocks} blocks, wall clock 100 MHz)")
