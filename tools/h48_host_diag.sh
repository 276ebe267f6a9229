#!/bin/bash
# GPU box: the host share seen by the process (cgroup CPU quota, throttling
# counters around each run) and H48 under several host pool sizes.
set -o pipefail
mkdir -p gpurun_out
echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "cpuset: $(cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null)"
nproc
for th in 16 8 16 4; do
  before=$(grep -E "nr_throttled|throttled_usec|usage_usec" /sys/fs/cgroup/cpu.stat 2>/dev/null | tr '\n' ' ')
  MSGPU_HOST_THREADS=$th timeout -k 10 200 python bench.py --config H48 --no-cpu --points= --fir-points= \
    --steps 50 --from-dicts-steps 0 --iso-steps 1 > gpurun_out/r06r_h48_t$th.json 2> gpurun_out/r06r_h48_t$th.log || exit $?
  after=$(grep -E "nr_throttled|throttled_usec|usage_usec" /sys/fs/cgroup/cpu.stat 2>/dev/null | tr '\n' ' ')
  python3 -c "
import json; d=json.load(open('gpurun_out/r06r_h48_t$th.json')); s=d['stage_ms']
print('threads $th', d['ms_per_step'], {k: s.get(k) for k in ('host_prep','host_plan_wall','host_records_wall','host_upload_wall')})"
  echo "  before: $before"; echo "  after:  $after"
done
