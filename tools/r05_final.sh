#!/bin/bash
# round-5 closing set: smoke, GPU suite + default bench (gpu_round.sh), then the profile set (prof_round.sh)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05z9_smoke.txt 2>&1 || { cat gpurun_out/r05z9_smoke.txt; exit 1; }
cat gpurun_out/r05z9_smoke.txt | tail -2
bash tools/gpu_round.sh r05z9 || exit $?
bash tools/prof_round.sh r05z9p
