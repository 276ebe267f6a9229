#!/bin/bash
# GPU box: persistent k_fir8 with the next segment loaded into registers during
# the epilogue (MSGPU_FIR8P=3) against the default (1): bit-identity test, C3 A/B.
set -o pipefail
mkdir -p gpurun_out
env MSGPU_FIR8P=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_long_filters.py -m gpu -q -x --timeout 200 \
  --timeout-method thread -k "fir8_persistent" > gpurun_out/r04t_tests.txt 2>&1 || { tail -20 gpurun_out/r04t_tests.txt; exit 1; }
tail -1 gpurun_out/r04t_tests.txt
run() {  # tag, env, args...
  local t=$1 e=$2; shift 2
  env MSGPU_FIR8P=$e timeout -k 10 300 python3 bench.py --no-cpu --from-dicts-steps 0 --points= "$@" \
    > gpurun_out/r04t_$t.json 2> gpurun_out/r04t_$t.log || exit $?
  python3 - gpurun_out/r04t_$t.json $t <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
i = d.get("roofline_isolated") or {}
print(sys.argv[2], "step", d["ms_per_step"], "ok", d["checked"]["all_ok"], "fir window", d["stage_ms"].get("fir_kernel"),
      "iso fir", (i.get("stage_ms") or {}).get("fir_kernel"), "iso total", (i.get("stage_ms") or {}).get("total"))
PY
}
for r in a b; do
  run C3_p3$r 3 --config C3 --steps 30
  run C3_p1$r 1 --config C3 --steps 30
done
run C5_p3 3 --config C5 --steps 3 --iso-steps 0 --gate none
