#!/bin/bash
# GPU box: GPU suite, then
# the default bench line, kernel stats + PMC traffic and SQ counters.
set -o pipefail
tag=${1:-r03ah}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.txt 2>&1
rc=$?
echo "== suite rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/${tag}_gpu_tests.txt | tail -4
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/${tag}_bench.json || exit $?
python3 - gpurun_out/${tag}_bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); i = d["roofline_isolated"]["stage_ms"]
print("C3 step", d["ms_per_step"], "value", d["value"], "ok", d["checked"]["all_ok"], "cpu", d["cpu_baseline"] and d["cpu_baseline"]["value"])
print("  iso", {k: i[k] for k in ("generate", "spectral", "overlap_add", "fir_kernel", "fir_h", "stereo", "total")})
for k, v in d["points"].items():
    print(k, "step", v["ms_per_step"], "value", v["value"], "check", (v["check"] or {}).get("all_ok"))
PY
BATCH=341 bash tools/profile.sh $tag > /dev/null 2>&1 || exit $?
bash tools/pmc_sq2.sh $tag || exit $?
python3 - $tag <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/{sys.argv[1]}_prof/**/*kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e6, 4), round(float(r["Percentage"]), 2))
PY
grep -A22 "^k_fir8<0>" gpurun_out/${tag}_sq_summary.txt | grep -E "INSTS_VALU|BANK|IDX_ACTIVE|insts per"
cat gpurun_out/${tag}_agree.txt
