#!/bin/bash
# Run GPU steps in order on the gpurun box, each under its own time limit.
# A test failure (exit 1) lets the next step run; a crash, abort, fault or
# timeout (any other non-zero code) stops the script so nothing else touches
# the GPU.   usage: tools/gpu_steps.sh SECONDS 'cmd1' [SECONDS 'cmd2' ...]
mkdir -p gpurun_out
while [ $# -ge 2 ]; do
  lim=$1; cmd=$2; shift 2
  echo "=== [$(date +%T)] ($lim s) $cmd"
  timeout -k 10 "$lim" bash -c "$cmd"
  rc=$?
  echo "=== rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal exit $rc: stopping"; exit $rc; fi
done
exit 0
