#!/bin/bash
# GPU box: full GPU suite on the product library, then FIR twiddle variants
# (tw0: powers, tw1: table everywhere, base: table for radix 16) on the
# long-filter tests and the C3 bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -v -s --timeout 200 --timeout-method thread \
  > gpurun_out/r03f_gpu_tests.txt 2>&1
rc=$?
echo "== full suite rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r03f_gpu_tests.txt | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in base tw0 tw1; do
  if [ "$v" != base ]; then export MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_$v.so; else unset MSGPU_LIB; fi
  timeout -k 10 200 python -u -m pytest tests/test_gpu_long_filters.py -v -s --timeout 200 --timeout-method thread \
    -k "long_space or fir8" > gpurun_out/r03f_${v}_tests.txt 2>&1
  echo "== $v"; grep -E "^ERIR|^ER384|MSGPU_FIR8=1|passed|failed" gpurun_out/r03f_${v}_tests.txt | tail -12
  timeout -k 10 200 python bench.py --no-cpu --points= --steps 20 > gpurun_out/r03f_${v}_bench.json || exit $?
  python3 - "$v" "gpurun_out/r03f_${v}_bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[2])); i = d["roofline_isolated"]["stage_ms"]; t = d["stage_ms"]
print(sys.argv[1], "step", d["ms_per_step"], "value", d["value"], "ok", d["checked"]["all_ok"])
print("  iso", {k: i[k] for k in ("generate", "spectral", "overlap_add", "fir_kernel", "fir_h", "stereo", "total")})
PY
done
