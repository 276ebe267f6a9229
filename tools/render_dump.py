#!/usr/bin/env python3
"""Render a config's batch with the library MSGPU_LIB names (default: the product
library) and save the output, for bit-identity checks between library builds.

    python tools/render_dump.py CONFIG BATCH OUT.npy
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-suite_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import msgpu  # noqa: E402
from msgpu.engine import Engine  # noqa: E402
from msgpu.pack import PackedBatch  # noqa: E402

cfg, batch, out_path = sys.argv[1], int(sys.argv[2]), sys.argv[3]
irs = bench.load_irs()
packed = PackedBatch([msgpu.config_params(cfg, seed=1000 + b, irs=irs) for b in range(batch)])
eng = Engine(0)
out = eng.render_packed(packed)
eng.torch.cuda.synchronize()
np.save(out_path, out.cpu().numpy())
print(cfg, batch, "frames", int(packed.total_frames), "->", out_path)
