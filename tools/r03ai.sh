#!/bin/bash
# GPU box: the ER merge's radix tap sort (product) against std::sort
# (libmsgpu_sort.so, MSG_TAP_RADIX=0) on the host-bound H48 point and on C3,
# alternating; then the GPU suite.
set -o pipefail
mkdir -p gpurun_out
for cfg in H48 C3; do
  for v in base sort base sort; do
    if [ "$v" != base ]; then export MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_$v.so; else unset MSGPU_LIB; fi
    timeout -k 10 200 python bench.py --config $cfg --no-cpu --iso-steps 1 --points= --steps 30 > gpurun_out/r03ai_${cfg}_$v.json 2>/dev/null || exit $?
    python3 -c "
import json;d=json.load(open('gpurun_out/r03ai_${cfg}_$v.json'));t=d['stage_ms']
print('$cfg', '$v', 'step', d['ms_per_step'], 'value', d['value'], 'ok', d['checked']['all_ok'], {k: t[k] for k in ('host_plan_wall','host_records_wall','host_upload_wall','host_preset_records','host_event_records')})"
  done
done
unset MSGPU_LIB
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r03ai_gpu_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/r03ai_gpu_tests.txt; exit $rc
