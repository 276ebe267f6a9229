#!/bin/bash
# GPU box: CU partition A/B on C3.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 bash tools/cusplit_ab.sh -,0,3 16,0x108:18,3 16,0x108:16,3 16,0x108:20,3 16,0x128:18,3 16,0x108:18,2 -,0x108:18,3 16,0,3 16,0x108:22,3 -,0,3 2>&1 || exit $?
