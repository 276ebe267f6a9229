#!/bin/bash
# GPU box: FIR accuracy and speed, table twiddles (product) vs powers (libmsgpu_twpow.so).
set -o pipefail
mkdir -p gpurun_out
for v in base twpow; do
  if [ "$v" != base ]; then export MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_$v.so; else unset MSGPU_LIB; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_long_filters.py tests/test_gpu_parity.py tests/test_gpu_fir.py \
    -v -s --timeout 200 --timeout-method thread > gpurun_out/r03e_${v}_tests.txt 2>&1
  rc=$?
  echo "== $v tests rc=$rc"
  grep -E "FAILED|passed|failed|MSGPU_FIR8=1|fir case|ERIR|ER384|^case 2 \[" gpurun_out/r03e_${v}_tests.txt | tail -22
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  timeout -k 10 200 python bench.py --no-cpu --points= --steps 20 > gpurun_out/r03e_${v}_bench.json || exit $?
  python3 - "$v" "gpurun_out/r03e_${v}_bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[2])); i = d["roofline_isolated"]["stage_ms"]; t = d["stage_ms"]
print(sys.argv[1], "step", d["ms_per_step"], "value", d["value"], "ok", d["checked"]["all_ok"])
print("  iso", {k: i[k] for k in ("generate", "spectral", "overlap_add", "fir_kernel", "fir_h", "stereo", "total")})
print("  timed", {k: t[k] for k in ("generate", "spectral", "overlap_add", "fir_kernel", "fir_h", "stereo")})
PY
done
