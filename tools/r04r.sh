#!/bin/bash
# GPU box: persistent k_fir8 without prefetch (MSGPU_FIR8P=1) against per-block (0), repeated.
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, env, args...
  local t=$1 e=$2; shift 2
  env MSGPU_FIR8P=$e timeout -k 10 300 python3 bench.py --no-cpu --from-dicts-steps 0 --points= "$@" \
    > gpurun_out/r04r_$t.json 2> gpurun_out/r04r_$t.log || exit $?
  python3 - gpurun_out/r04r_$t.json $t <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
i = d.get("roofline_isolated") or {}
print(sys.argv[2], "step", d["ms_per_step"], "ok", d["checked"]["all_ok"], "roof", d["roofline"]["kernel_ms"], d["roofline"]["frac"],
      "iso fir", (i.get("stage_ms") or {}).get("fir_kernel"), "iso total", (i.get("stage_ms") or {}).get("total"))
PY
}
for r in a b c; do
  run C3_p1$r 1 --config C3 --steps 30
  run C3_p0$r 0 --config C3 --steps 30
done
run C4_p1 1 --config C4 --steps 30 --iso-steps 0
run C4_p0 0 --config C4 --steps 30 --iso-steps 0
run C4_p1b 1 --config C4 --steps 30 --iso-steps 0
run C5_p1 1 --config C5 --steps 3 --iso-steps 0 --gate none
run C5_p0 0 --config C5 --steps 3 --iso-steps 0 --gate none
