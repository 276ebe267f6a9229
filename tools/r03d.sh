#!/bin/bash
# GPU box: k_fir8 parity + A/B, stage pins, then H48 with threaded vs serial enqueue.
set -o pipefail
bash tools/ab_fir8.sh r03d || exit $?
timeout -k 10 200 python -u -m pytest tests/test_gpu_stage_pins.py -v -s --timeout 120 --timeout-method thread \
  > gpurun_out/r03d_pins.txt 2>&1
grep -E "rel rms|passed|failed|FAILED|Error" gpurun_out/r03d_pins.txt | cut -c1-300 | tail -20
for e in threads serial; do
  timeout -k 10 200 python bench.py --no-cpu --config H48 --points= --steps 20 --iso-steps 0 --enqueue $e \
    > gpurun_out/r03d_h48_$e.json || exit $?
  python3 - "$e" "gpurun_out/r03d_h48_$e.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[2])); t = d["stage_ms"]
print("H48", sys.argv[1], "step", d["ms_per_step"], "value", d["value"],
      {k: t[k] for k in t if k.startswith("host")})
PY
done
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "progress or gated or two_engines" -v --timeout 120 --timeout-method thread 2>&1 | tail -6
