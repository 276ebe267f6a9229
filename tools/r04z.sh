#!/bin/bash
# GPU box: k_spec3's wide-band inverse pass 1 with compile-time twiddle ratios
# (MSG_S3_WIDE_TW=1, default) against per-input table twiddles (=0, experiment
# library): spec3 parity tests, C4 / C3 A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 200 --timeout-method thread \
  -k "spec3 or parity" > gpurun_out/${TAG:-r04z}_tests.txt 2>&1 || { grep -E "FAIL|Error|passed|failed" gpurun_out/${TAG:-r04z}_tests.txt | tail; exit 1; }
tail -n 1 gpurun_out/${TAG:-r04z}_tests.txt
run() {  # tag, lib, args...
  local t=$1 l=$2; shift 2
  env ${l:+MSGPU_LIB=$l} timeout -k 10 300 python3 bench.py --no-cpu --from-dicts-steps 0 --points= "$@" \
    > gpurun_out/${TAG:-r04z}_$t.json 2> gpurun_out/${TAG:-r04z}_$t.log || exit $?
  python3 - gpurun_out/${TAG:-r04z}_$t.json $t <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
i = d.get("roofline_isolated") or {}
print(sys.argv[2], "step", d["ms_per_step"], "ok", d["checked"]["all_ok"], "iso", {k: v for k, v in (i.get("stage_ms") or {}).items() if k in ("generate", "spectral", "fir_kernel", "stereo", "total")})
PY
}
T0=audio-suite_amd/msgpu/libmsgpu_tw0.so
run C4_tw1a "" --config C4 --steps 30
run C4_tw0a $T0 --config C4 --steps 30
run C4_tw1b "" --config C4 --steps 30
run C4_tw0b $T0 --config C4 --steps 30
