#!/usr/bin/env python3
"""Time the LDS FFT engine alone (msg_bench_fft): forward+inverse real transforms."""
import ctypes as C
import math
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-suite_amd"))
from msgpu import _lib as L  # noqa: E402
from msgpu.engine import Engine  # noqa: E402

eng = Engine(0)
lib = L.lib()
for n in [int(a) for a in sys.argv[1:]] or [32768, 37500, 2400, 1920, 16384, 8192]:
    for reps in (4,):
        blocks = 2048
        ms = C.c_float(0)
        L.check(lib.msg_bench_fft(eng._ctx, n, reps, blocks, C.byref(ms)), eng._ctx)
        per = ms.value * 1e3 / (2 * reps * blocks / 256)   # us per transform per CU
        flops = 2.5 * n * math.log2(n)
        print(f"n={n:6d}: {ms.value:8.3f} ms for {2*reps*blocks} transforms -> {per:7.2f} us/transform/CU, "
              f"{2*reps*blocks*flops/ms.value/1e9:7.1f} GFLOP/s")
