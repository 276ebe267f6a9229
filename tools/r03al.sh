#!/bin/bash
# GPU box: the final round-3 library -- smoke(), the GPU suite, the default
# bench line, kernel stats, PMC traffic and SQ counters.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03al_smoke.txt 2>&1 || exit $?
cat gpurun_out/r03al_smoke.txt
bash tools/gpu_full.sh r03al
