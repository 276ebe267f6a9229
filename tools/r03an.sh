#!/bin/bash
# GPU box: H48 (host-bound) sub-batch size x streams x gate sweep, two rounds
# alternating, 20 steps each; the default is 3 streams, 341 presets, gate 2,4.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r03an_h48_sweep.txt; : > $out
for round in 1 2; do
  for cfg in "3 341 2,4" "3 341 none" "3 171 2,4" "3 171 none" "3 128 none" "2 512 2,4" "2 256 none" "4 256 none" "4 128 none"; do
    set -- $cfg
    timeout -k 10 120 python bench.py --config H48 --no-cpu --iso-steps 0 --points= --steps 20 \
        --streams $1 --sub $2 --gate $3 > gpurun_out/r03an_tmp.json 2>/dev/null || { echo "fail $cfg" >> $out; continue; }
    python3 -c "
import json;d=json.load(open('gpurun_out/r03an_tmp.json'));t=d['stage_ms']
print('round $round streams $1 sub $2 gate $3', 'step', d['ms_per_step'], 'value', round(d['value']), 'ok', d['checked']['all_ok'], 'plan', t['host_plan_wall'], 'rec', t['host_records_wall'], 'up', t['host_upload_wall'])" >> $out
  done
done
cat $out
