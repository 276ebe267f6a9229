#!/bin/bash
# A/B of in-flight sub-batches per GPU (contexts/streams) and stream gates on
# the default bench workload.   usage (on the box): bash tools/streams_ab.sh "ARGS" ["ARGS" ...]
#   e.g. bash tools/streams_ab.sh "--streams 2 --gate 2,4" "--streams 3 --gate 2,4"
set -e
mkdir -p gpurun_out
for a in "$@"; do
  timeout -k 10 200 python bench.py --no-cpu --points= $a > gpurun_out/st.json 2>/dev/null
  python3 -c "
import json;d=json.load(open('gpurun_out/st.json'));print('$a', d['ms_per_step'], d['value'], d['checked']['all_ok'])"
done
