#!/bin/bash
# A/B of stream count x gate schedule on the default C3 bench workload (no CPU
# baseline, no points), in alternating order.
#   usage (on the box): bash tools/sched_ab.sh "3 2,4" "3 none" "4 2,4" ...
set -e
mkdir -p gpurun_out
for cfg in "$@"; do
  set -- $cfg
  s=$1; g=$2; tag="s${s}_g${g/,/_}"
  timeout -k 10 200 python bench.py --no-cpu --points= --iso-steps 0 --streams "$s" --gate "$g" > gpurun_out/sched_$tag.json 2>/dev/null
  python3 -c "
import json;d=json.load(open('gpurun_out/sched_$tag.json'))
print('streams $s gate $g', 'step', d['ms_per_step'], 'Msamples/s', d['value'], 'ok', d['checked']['all_ok'])"
done
