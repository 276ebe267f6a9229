#!/bin/bash
# (MSGPU_CU_SPLIT lived in a tuning build only: profiles/r03ag_cusplit_ab.json.)
# A/B of a CU partition between the stages (tuning build with MSGPU_CU_SPLIT)
# on C3.  spec = QUEUES,SPLIT,STREAMS (QUEUES: GPU_MAX_HW_QUEUES, '-' = default;
# SPLIT: MSGPU_CU_SPLIT "STAGES:K" or 0 = none; STREAMS: bench --streams)
#   usage (on the box): bash tools/cusplit_ab.sh SPEC [SPEC ...]
set -e
mkdir -p gpurun_out
for v in "$@"; do
  IFS=, read -r q sp st <<< "$v"
  unset MSGPU_CU_SPLIT GPU_MAX_HW_QUEUES
  [ "$q" != - ] && export GPU_MAX_HW_QUEUES=$q
  [ "$sp" != 0 ] && export MSGPU_CU_SPLIT=$sp
  f=gpurun_out/cusplit_$(echo "$v" | tr ',:' '__').json
  timeout -k 10 200 python bench.py --no-cpu --points= --streams $st > $f 2>/dev/null
  python3 -c "
import json;d=json.load(open('$f'))
print('$v', 'step', d['ms_per_step'], 'ok', d['checked']['all_ok'])"
done
