#!/bin/bash
# (The MSGPU_PRIO_* knob lived in a tuning build only: profiles/r03af_queues_prio_ab.json.)
# A/B of hardware queues x stage stream priorities x streams on C3.
#   spec = QUEUES,HI,LO,STREAMS (QUEUES: GPU_MAX_HW_QUEUES, '-' = default;
#   HI/LO: MSGPU_PRIO_HI/LO stage masks, 0 = none; STREAMS: bench --streams)
#   usage (on the box): bash tools/prio_ab2.sh SPEC [SPEC ...]
set -e
mkdir -p gpurun_out
for v in "$@"; do
  IFS=, read -r q hi lo st <<< "$v"
  unset MSGPU_PRIO_HI MSGPU_PRIO_LO GPU_MAX_HW_QUEUES
  [ "$q" != - ] && export GPU_MAX_HW_QUEUES=$q
  [ "$hi" != 0 ] && export MSGPU_PRIO_HI=$hi
  [ "$lo" != 0 ] && export MSGPU_PRIO_LO=$lo
  f=gpurun_out/prio2_${v//,/_}.json
  timeout -k 10 200 python bench.py --no-cpu --points= --streams $st > $f 2>/dev/null
  python3 -c "
import json;d=json.load(open('$f'))
print('$v', 'step', d['ms_per_step'], 'ok', d['checked']['all_ok'])"
done
