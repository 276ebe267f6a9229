#!/bin/bash
# GPU box: persistent k_fir8 (MSGPU_FIR8P = 0 per-block, 1 persistent, 2 persistent
# + L2 prefetch): bit-identity and parity tests, then C3 / C4 / C5 A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_long_filters.py -m gpu -v -s --timeout 200 --timeout-method thread \
  -k "fir8 or fir64 or long_space" > gpurun_out/r04q_tests.txt 2>&1 || { tail -30 gpurun_out/r04q_tests.txt; exit 1; }
grep -E "passed|failed" gpurun_out/r04q_tests.txt | tail -2
run() {  # tag, env, args...
  local t=$1 e=$2; shift 2
  env MSGPU_FIR8P=$e timeout -k 10 300 python3 bench.py --no-cpu --from-dicts-steps 0 --points= "$@" \
    > gpurun_out/r04q_$t.json 2> gpurun_out/r04q_$t.log || exit $?
  python3 - gpurun_out/r04q_$t.json $t <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
i = d.get("roofline_isolated") or {}
print(sys.argv[2], "step", d["ms_per_step"], "ok", d["checked"]["all_ok"], "roof", d["roofline"]["kernel_ms"], d["roofline"]["frac"],
      "iso fir", (i.get("stage_ms") or {}).get("fir_kernel"), "iso total", (i.get("stage_ms") or {}).get("total"))
PY
}
run C3_p0 0 --config C3 --steps 20
run C3_p2 2 --config C3 --steps 20
run C3_p1 1 --config C3 --steps 20
run C3_p2b 2 --config C3 --steps 20
run C3_p0b 0 --config C3 --steps 20
run C4_p0 0 --config C4 --steps 30 --iso-steps 0
run C4_p2 2 --config C4 --steps 30 --iso-steps 0
run C5_p0 0 --config C5 --steps 3 --iso-steps 0 --gate none
run C5_p2 2 --config C5 --steps 3 --iso-steps 0 --gate none
