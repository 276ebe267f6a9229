#!/bin/bash
# GPU box: full GPU suite, C3 bench, kernel stats.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread \
  > gpurun_out/r03h_gpu_tests.txt 2>&1
rc=$?
echo "== full suite rc=$rc"; grep -E "FAILED|passed|failed|^ERIR|^ER384|MSGPU_FIR8=1" gpurun_out/r03h_gpu_tests.txt | tail -14
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu --points=H48,C4,C5 --steps 20 --point-steps 10 > gpurun_out/r03h_bench.json || exit $?
python3 - gpurun_out/r03h_bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); i = d["roofline_isolated"]["stage_ms"]; t = d["stage_ms"]
print("C3 step", d["ms_per_step"], "value", d["value"], "ok", d["checked"]["all_ok"])
print("  iso", {k: i[k] for k in ("generate", "spectral", "overlap_add", "fir_kernel", "fir_h", "stereo", "total")})
for k, v in d["points"].items():
    print(k, "step", v["ms_per_step"], "value", v["value"], "check", (v["check"] or {}).get("all_ok"))
PY
BATCH=341 bash tools/profile.sh r03h > /dev/null 2>&1 || exit $?
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r03h_prof/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e6, 4), round(float(r["Percentage"]), 2))
PY
