#!/bin/bash
# GPU box: k_fir8 parity tests, then the C3 bench with k_fir8 on and off.
#   bash tools/ab_fir8.sh TAG
set -o pipefail
tag=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_long_filters.py tests/test_gpu_parity.py tests/test_gpu_fir.py \
  -v -s --timeout 200 --timeout-method thread > gpurun_out/${tag}_gpu_tests.txt 2>&1
rc=$?
grep -E "FAILED|passed|failed|MSGPU_FIR8|fir case|^case|ERIR|ER384" gpurun_out/${tag}_gpu_tests.txt | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for f in 1 0; do
  MSGPU_FIR8=$f timeout -k 10 200 python bench.py --no-cpu --points= --steps 20 > gpurun_out/${tag}_bench_fir8_$f.json || exit $?
  python3 - "$f" "gpurun_out/${tag}_bench_fir8_$f.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[2])); i = d["roofline_isolated"]["stage_ms"]; t = d["stage_ms"]
print("fir8=" + sys.argv[1], "step", d["ms_per_step"], "ok", d["checked"]["all_ok"],
      "iso", {k: i[k] for k in ("fir_kernel", "fir_h", "total")}, "timed", {k: t[k] for k in ("fir_kernel", "fir_h")})
PY
done
