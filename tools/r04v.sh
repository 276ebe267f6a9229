#!/bin/bash
# GPU box: k_spec3's 960-point plan for C5's grains (MSGPU_S3_960=0 keeps them on
# k_spectral_ct): parity tests, C5 A/B, then the schedule sweep with the
# persistent FIR (tools/r04u.sh).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long_filters.py -m gpu -v -s --timeout 200 \
  --timeout-method thread -k "spec3 or fir8_persistent" > gpurun_out/r04v_tests.txt 2>&1 || { grep -E "FAIL|Error|passed|failed" gpurun_out/r04v_tests.txt | tail -20; exit 1; }
grep -E "C5|passed|failed" gpurun_out/r04v_tests.txt | tail -12
run() {  # tag, env, args...
  local t=$1 e=$2; shift 2
  env MSGPU_S3_960=$e timeout -k 10 300 python3 bench.py --no-cpu --from-dicts-steps 0 --points= "$@" \
    > gpurun_out/r04v_$t.json 2> gpurun_out/r04v_$t.log || exit $?
  python3 - gpurun_out/r04v_$t.json $t <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
i = d.get("roofline_isolated") or {}
print(sys.argv[2], "step", d["ms_per_step"], "ok", d["checked"]["all_ok"], "iso", {k: v for k, v in (i.get("stage_ms") or {}).items() if k in ("generate", "spectral", "fir_kernel", "stereo", "total")})
PY
}
run C5_s1 1 --config C5 --steps 3 --gate none
run C5_s0 0 --config C5 --steps 3 --gate none
run C5_s1b 1 --config C5 --steps 3 --gate none
