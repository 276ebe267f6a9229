#!/bin/bash
# GPU box: table copies with every load in flight before the LDS stores
# (TabCopy, MSG_TAB_PRELOAD=1, product) against the per-iteration copy loop
# (libmsgpu_old.so: k_fir + k_spec3 TUs with MSG_TAB_PRELOAD=0), then the
# full suite, bench line, kernel stats, PMC traffic and SQ counters.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 bash tools/lib_ab.sh base old base old > gpurun_out/r03ah_ab.txt 2>&1 || exit $?
cat gpurun_out/r03ah_ab.txt
bash tools/gpu_full.sh r03ah
