#!/bin/bash
# GPU box: H48 after 3 or 30 warmup steps, stage events every batch or none, alternating.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for cfg in "3 1" "30 1" "3 0" "30 0"; do
    set -- $cfg
    MSGPU_BENCH_PROFILE_EVERY=$2 timeout -k 10 200 python bench.py --config H48 --no-cpu --points= --fir-points= \
      --steps 50 --warmup $1 --from-dicts-steps 0 --iso-steps 0 > gpurun_out/r06wu_$1_$2_$i.json 2> gpurun_out/r06wu_$1_$2_$i.log || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r06wu_$1_$2_$i.json'))
print('H48 warmup $1 every $2', $i, d['ms_per_step'], d['checked']['all_ok'])"
  done
done
