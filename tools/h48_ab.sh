#!/bin/bash
# GPU box: H48 (host-bound) A/B of library builds, alternating, two rounds.
#   usage: bash tools/h48_ab.sh TAG lib_a.so lib_b.so ...   (names under audio-suite_amd/msgpu/)
set -o pipefail
tag=${1:?tag}; shift
mkdir -p gpurun_out
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"
grep -m1 'model name' /proc/cpuinfo
for i in 1 2; do
 for lib in "$@"; do
  out=gpurun_out/${tag}_${lib%.so}_$i
  MSGPU_LIB=audio-suite_amd/msgpu/$lib timeout -k 10 200 python bench.py --config H48 --no-cpu --points= --fir-points= \
    --steps 50 --from-dicts-steps 0 --iso-steps 1 > $out.json 2> $out.log || exit $?
  python3 -c "
import json; d=json.load(open('$out.json')); s=d['stage_ms']
print('$lib', $i, d['ms_per_step'], d['checked']['all_ok'], {k: s.get(k) for k in ('host_prep','host_plan_wall','host_records_wall','host_upload_wall','host_plan_sizes','host_plan_events','host_preset_records','host_event_records')})"
 done
done
