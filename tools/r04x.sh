#!/bin/bash
# GPU box: the resonant emission from bases at multiples of 64 (MSG_GEN_EMIT=3,
# default) against the per-group bases (=2, experiment library): GPU suite, then
# C3 / C5 A/B of the generate stage.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread \
  > gpurun_out/r04x_gpu_tests.txt 2>&1; rc=$?
grep -E "FAILED|passed|failed" gpurun_out/r04x_gpu_tests.txt | tail -8
grep -E "micro rel err" gpurun_out/r04x_gpu_tests.txt | head -4
if [ $rc -gt 1 ]; then exit $rc; fi
run() {  # tag, lib, args...
  local t=$1 l=$2; shift 2
  env ${l:+MSGPU_LIB=$l} timeout -k 10 300 python3 bench.py --no-cpu --from-dicts-steps 0 --points= "$@" \
    > gpurun_out/r04x_$t.json 2> gpurun_out/r04x_$t.log || exit $?
  python3 - gpurun_out/r04x_$t.json $t <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
i = d.get("roofline_isolated") or {}
print(sys.argv[2], "step", d["ms_per_step"], "ok", d["checked"]["all_ok"], "iso", {k: v for k, v in (i.get("stage_ms") or {}).items() if k in ("generate", "spectral", "fir_kernel", "stereo", "total")})
PY
}
E2=audio-suite_amd/msgpu/libmsgpu_emit2.so
run C3_e3a "" --config C3 --steps 30
run C3_e2a $E2 --config C3 --steps 30
run C3_e3b "" --config C3 --steps 30
run C3_e2b $E2 --config C3 --steps 30
run C5_e3 "" --config C5 --steps 3 --gate none
run C5_e2 $E2 --config C5 --steps 3 --gate none
runc() {  # tag, cus, args...
  local t=$1 c=$2; shift 2
  env MSGPU_FIR8P_CUS=$c timeout -k 10 300 python3 bench.py --no-cpu --from-dicts-steps 0 --points= --iso-steps 0 "$@" \
    > gpurun_out/r04x_$t.json 2> gpurun_out/r04x_$t.log || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04x_$t.json')); print('$t', d['ms_per_step'], d['checked']['all_ok'], 'fir window', d['stage_ms'].get('fir_kernel'))"
}
runc C3_cu192 192 --config C3 --steps 30
runc C3_cu128 128 --config C3 --steps 30
runc C3_cu256 256 --config C3 --steps 30
runc C5_cu192 192 --config C5 --steps 3 --gate none
