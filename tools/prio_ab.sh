#!/bin/bash
# A/B of stage stream priorities (MSGPU_PRIO_HI / MSGPU_PRIO_LO stage masks:
# (The MSGPU_PRIO_HI / MSGPU_PRIO_LO knob lived in a tuning build only and was
# removed after this A/B: profiles/r03ad_prio_ab.json, r03af_queues_prio_ab.json.)
# 0x4 generate, 0x8 spectral, 0x10 overlap-add, 0x20 h build, 0x100 FIR, 0x40 stereo).
#   usage (on the box): bash tools/prio_ab.sh base HI:LO [HI:LO ...]
set -e
mkdir -p gpurun_out
for v in "$@"; do
  unset MSGPU_PRIO_HI MSGPU_PRIO_LO
  if [ "$v" != base ]; then export MSGPU_PRIO_HI=${v%%:*} MSGPU_PRIO_LO=${v##*:}; fi
  timeout -k 10 200 python bench.py --no-cpu --points= > gpurun_out/prio_$v.json 2>/dev/null
  python3 -c "
import json;d=json.load(open('gpurun_out/prio_$v.json'))
print('$v', 'step', d['ms_per_step'], 'ok', d['checked']['all_ok'])"
done
