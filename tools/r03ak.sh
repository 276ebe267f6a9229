#!/bin/bash
# GPU box: traversal order against the Infinity Cache -- k_ola_env and
# k_stereo_max walking their jobs backwards (rev: both, revst: stereo max
# only) against the forward product, alternating; then one FETCH_SIZE pass per
# library (HBM read bytes per kernel).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 bash tools/lib_ab.sh base rev revst base rev revst > gpurun_out/r03ak_ab.txt 2>&1; rc=$?
cat gpurun_out/r03ak_ab.txt; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
R=$PWD
for v in base rev; do
  if [ "$v" != base ]; then export MSGPU_LIB=$R/audio-suite_amd/msgpu/libmsgpu_$v.so; else unset MSGPU_LIB; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/r03ak_fetch_$v" -o run -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --iso-steps 0 --points= > "$R/gpurun_out/r03ak_fetch_$v.log" 2>&1) || exit $?
done
unset MSGPU_LIB
python3 - <<'PY'
import csv, glob, collections
for v in ("base", "rev"):
    f = glob.glob(f"gpurun_out/r03ak_fetch_{v}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName")
        acc[k[:24]][0] += float(r["Counter_Value"]); acc[k[:24]][1] += 1
    print(v, {k: round(s / n / 1024, 1) for k, (s, n) in acc.items() if any(x in k for x in ("ola", "stereo", "fir8<", "spec3"))}, "MB per launch (FETCH_SIZE KB/1024)")
PY
