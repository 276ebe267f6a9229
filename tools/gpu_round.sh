#!/bin/bash
# GPU box: the GPU suite (all failures listed), then the default bench
# line when the suite ended normally (pass or test failures, no fault/timeout).
set -o pipefail
tag=${1:?usage: tools/gpu_round.sh TAG}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.txt 2>&1
rc=$?
echo "== suite rc=$rc"; grep -E "FAILED|passed|failed|Error" gpurun_out/${tag}_gpu_tests.txt | tail -12
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.log || exit $?
python3 - gpurun_out/${tag}_bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("C3 step", d["ms_per_step"], "value", d["value"], "ok", d["checked"]["all_ok"], "roof", d["roofline"]["kernel"], d["roofline"]["frac"])
i = d["roofline_isolated"]
print("  iso", {k: i["stage_ms"][k] for k in ("generate", "spectral", "overlap_add", "fir_kernel", "fir_h", "stereo", "total")}, i.get("kernels_frac"))
print("  from_dicts", d.get("from_dicts") or d.get("points", {}).get("C3", {}).get("from_dicts"))
for k, v in d["points"].items():
    iso = v.get("roofline_isolated") or {}
    if k.startswith("FIR"):
        print(k, "step", v["ms_per_step"], "value", v["value"], "shape", v["fir_shape"], "roof", v["roofline"]["frac"],
              v["roofline"]["kernel_ms"], "check", v["check"])
        continue
    print(k, "step", v["ms_per_step"], "value", v["value"], "check", (v["check"] or {}).get("all_ok"),
          "iso", {a: b for a, b in (iso.get("stage_ms") or {}).items() if a in ("generate", "spectral", "overlap_add", "fir_kernel", "stereo", "total")},
          "fd", v.get("from_dicts"))
print("cpu", d["cpu_baseline"])
print("summary", json.dumps(d.get("points_summary")))
PY
