#!/bin/bash
# GPU box: hardware queues x stage priorities A/B on C3.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 bash tools/prio_ab2.sh -,0,0,3 8,0,0,3 -,0x108,0,2 -,0,0,2 8,0x108,0,3 8,0,0x4,3 16,0x108,0x4,3 8,0x8,0,3 8,0x100,0,3 -,0,0,3 8,0,0,3 8,0x108,0,3 2>&1 || exit $?
