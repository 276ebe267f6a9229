#!/bin/bash
# GPU box: k_spec3 library A/B.  usage: bash tools/s3_ab.sh TAG OLD NEW
#   OLD / NEW: library names libmsgpu_<name>.so, "base" = the product library;
#   stamps libraries libmsgpu_st<name>.so when present.
# Bit identity on C3 / C4 batches, spec3 parity tests, phase stamps, then
# alternating C4 and C3 bench runs.
set -o pipefail
tag=$1; old=$2; new=$3
mkdir -p gpurun_out
L=$PWD/audio-suite_amd/msgpu
lib() { if [ "$1" = base ]; then echo ""; else echo "$L/libmsgpu_$1.so"; fi; }
for c in C3 C4; do
  for v in $old $new; do
    MSGPU_LIB=$(lib $v) timeout -k 10 200 python tools/render_dump.py $c 64 /tmp/${tag}_${c}_$v.npy > /dev/null || exit $?
  done
  python3 -c "
import numpy as np
a=np.load('/tmp/${tag}_${c}_$old.npy'); b=np.load('/tmp/${tag}_${c}_$new.npy')
print('$c bit-identical', np.array_equal(a,b), 'max abs diff', float(np.abs(a-b).max()))"
done
rm -f /tmp/${tag}_*.npy
MSGPU_LIB=$(lib $new) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_long_filters.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.txt 2>&1 || { tail -20 gpurun_out/${tag}_tests.txt; exit 1; }
tail -1 gpurun_out/${tag}_tests.txt
for v in $old $new; do
  if [ -f $L/libmsgpu_st$v.so ]; then
    for c in C3 C4; do
      MSGPU_LIB=$L/libmsgpu_st$v.so timeout -k 10 200 python tools/spec3_stamps.py $c 171 > gpurun_out/${tag}_st_${v}_$c.txt 2>&1 || exit $?
      echo "== stamps $v $c"; grep -v amdgpu.ids gpurun_out/${tag}_st_${v}_$c.txt
    done
  fi
done
run() {  # tag lib args...
  local t=$1 v=$2; shift 2
  MSGPU_LIB=$(lib $v) timeout -k 10 300 python3 bench.py --no-cpu --from-dicts-steps 0 --points= "$@" > gpurun_out/${tag}_$t.json 2> gpurun_out/${tag}_$t.log || exit $?
  python3 - gpurun_out/${tag}_$t.json $t <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
i = (d.get("roofline_isolated") or {}).get("stage_ms") or {}
print(sys.argv[2], "step", d["ms_per_step"], "ok", d["checked"]["all_ok"], "iso spectral", i.get("spectral"), "iso total", i.get("total"))
PY
}
run C4_old $old --config C4 --steps 30
run C4_new $new --config C4 --steps 30
run C3_old $old --config C3 --steps 20
run C3_new $new --config C3 --steps 20
run C4_old2 $old --config C4 --steps 30
run C4_new2 $new --config C4 --steps 30
run C3_old2 $old --config C3 --steps 20
run C3_new2 $new --config C3 --steps 20
