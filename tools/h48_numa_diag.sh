#!/bin/bash
# GPU box: where the GPU sits (PCI device -> NUMA node, local CPUs) and H48 with
# the process pinned to 16 GPU-local CPUs, 16 CPUs of the other node, or unpinned.
set -o pipefail
mkdir -p gpurun_out
for d in /sys/class/drm/card*/device; do
  [ -e $d/numa_node ] && echo "$d numa $(cat $d/numa_node) local $(cat $d/local_cpulist 2>/dev/null) vendor $(cat $d/vendor) id $(cat $d/device)"
done
python3 - <<'PY'
import torch
p = torch.cuda.get_device_properties(0)
print("torch pci", getattr(p, "pci_bus_id", None), getattr(p, "pci_device_id", None), getattr(p, "pci_domain_id", None))
PY
lscpu | grep -E "NUMA|Socket|Thread|Core" || true
run() {
  tag=$1; shift
  timeout -k 10 200 "$@" python bench.py --config H48 --no-cpu --points= --fir-points= --steps 50 --from-dicts-steps 0 \
    --iso-steps 1 > gpurun_out/r06s_$tag.json 2> gpurun_out/r06s_$tag.log || return $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r06s_$tag.json')); s=d['stage_ms']
print('$tag', d['ms_per_step'], {k: s.get(k) for k in ('host_prep','host_plan_wall','host_records_wall','host_upload_wall')})"
}
read LOCAL REMOTE < <(python3 - <<'PY'
import os, torch
p = torch.cuda.get_device_properties(0)
addr = "%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
base = "/sys/bus/pci/devices/" + addr
def expand(s):
    out = []
    for part in s.strip().split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out
loc = expand(open(base + "/local_cpulist").read())
allc = sorted(os.sched_getaffinity(0))
rem = [c for c in allc if c not in set(loc)]
import sys
print(addr, open(base + "/numa_node").read().strip(), len(loc), len(rem), file=sys.stderr)
print(",".join(map(str, loc[:16])), ",".join(map(str, (rem or loc)[:16])))
PY
)
echo "local $LOCAL remote $REMOTE"
for i in 1 2; do
  run free$i env || exit 1
  run local$i taskset -c $LOCAL || exit 1
  run remote$i taskset -c $REMOTE || exit 1
done
