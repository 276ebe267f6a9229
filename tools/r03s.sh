#!/bin/bash
# GPU box: default bench line and kernel stats of the same workload (event-timed stage
# windows vs rocprofv3 kernel averages, after moving the gate wait before the stage event).
set -o pipefail
tag=r03s
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.txt 2>&1 || exit $?
tail -1 gpurun_out/${tag}_gpu_tests.txt
timeout -k 10 400 python bench.py --points=H48 > gpurun_out/${tag}_bench.json || exit $?
python3 - gpurun_out/${tag}_bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("C3 step", d["ms_per_step"], "value", d["value"], "roofline", d["roofline"]["kernel"], d["roofline"]["kernel_ms"], d["roofline"]["frac"])
print("  timed", {k: d["stage_ms"][k] for k in ("generate", "spectral", "overlap_add", "fir_kernel", "fir_h", "stereo")})
PY
BATCH=341 bash tools/profile.sh $tag > /dev/null 2>&1 || exit $?
python3 - $tag <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/{sys.argv[1]}_prof/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e6, 4), round(float(r["Percentage"]), 2))
PY
