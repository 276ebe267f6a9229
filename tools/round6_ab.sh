#!/bin/bash
# GPU box: the round-6 A/B and diagnostic sessions, one function each (their
# records are under profiles/r06*; DESIGN section 9 cites them).
#   usage (on the box): bash tools/round6_ab.sh NAME [args]
# NAME: c3_streams c3_streams32 h48_host_diag h48_numa_diag h48_sched gate_points_ab gate_c3_ab h48_streams_ab prof_every_ab prof_every_ab2 h48_warmup_ab sub_sweep s3p_check fir8_cus_stamps ho_check q2nt_ab mb_check c5_sub_ab q2_ahead1_ab
set -o pipefail
mkdir -p gpurun_out

# GPU box: the host share seen by the process (cgroup CPU quota, throttling
# counters around each run) and H48 under several host pool sizes.
h48_host_diag() {
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
}

# GPU box: where the GPU sits (PCI device -> NUMA node, local CPUs) and H48 with
# the process pinned to 16 GPU-local CPUs, 16 CPUs of the other node, or unpinned.
h48_numa_diag() {
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
}

# GPU box: H48's sub-batch size / stream count / gate (the step is a per-stream
# latency chain of ~20 small kernels, not throughput), alternating configurations.
h48_sched() {
run() {
  tag=$1; shift
  timeout -k 10 200 python bench.py --config H48 --no-cpu --points= --fir-points= --steps 50 --from-dicts-steps 0 \
    --iso-steps 0 "$@" > gpurun_out/r06h48s_$tag.json 2> gpurun_out/r06h48s_$tag.log || return $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r06h48s_$tag.json'))
print('$tag', '$*', d['ms_per_step'], d['checked']['all_ok'], d['config'].get('sub_batches_per_gpu'), d['config'].get('stream_gate'))"
}
for i in 1 2; do
  run base$i || exit 1
  run s171_$i --sub 171 || exit 1
  run s128_$i --sub 128 || exit 1
  run s256x4_$i --sub 256 --streams 4 || exit 1
  run s171x6_$i --sub 171 --streams 6 || exit 1
  run nogate$i --gate none || exit 1
done
}

# GPU box: the 2,4 stream gate against none on the short-step points (H48, C4),
# alternating, three pairs each.
gate_points_ab() {
run() {
  cfg=$1; tag=$2; shift 2
  timeout -k 10 200 python bench.py --config $cfg --no-cpu --points= --fir-points= --steps 50 --from-dicts-steps 0 \
    --iso-steps 0 "$@" > gpurun_out/r06g2_${cfg}_$tag.json 2> gpurun_out/r06g2_${cfg}_$tag.log || return $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r06g2_${cfg}_$tag.json'))
print('$cfg $tag', d['ms_per_step'], d['checked']['all_ok'], d['config'].get('stream_gate'))"
}
for cfg in H48 C4; do
  for i in 1 2 3; do
    run $cfg gate$i || exit 1
    run $cfg none$i --gate none || exit 1
  done
done
}

# GPU box: C3's stream gate re-measured on the round-6 kernels, alternating pairs.
gate_c3_ab() {
for i in 1 2 3; do
  for g in 2,4 none; do
    timeout -k 10 200 python bench.py --no-cpu --points= --fir-points= --steps 40 --from-dicts-steps 0 --iso-steps 0 \
      --gate $g > gpurun_out/r06g3_${g/,/_}_$i.json 2> gpurun_out/r06g3_${g/,/_}_$i.log || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r06g3_${g/,/_}_$i.json'))
print('C3 gate $g', $i, d['ms_per_step'], d['checked']['all_ok'])"
  done
done
}

# GPU box: H48 ungated with 2 / 3 / 4 streams (sub-batches of 512 / 341 / 256), alternating.
h48_streams_ab() {
for i in 1 2; do
  for cfg in "3 341" "2 512" "4 256"; do
    set -- $cfg
    timeout -k 10 200 python bench.py --config H48 --no-cpu --points= --fir-points= --steps 50 --from-dicts-steps 0 \
      --iso-steps 0 --gate none --streams $1 --sub $2 > gpurun_out/r06hs_$1_$i.json 2> gpurun_out/r06hs_$1_$i.log || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r06hs_$1_$i.json'))
print('H48 streams $1 sub $2', $i, d['ms_per_step'], d['checked']['all_ok'])"
  done
done
}

# GPU box: sampled stage profiling (bench PROFILE_EVERY = 4) -- H48 and C3 lines,
# and the stage-time GPU tests.
prof_every_ab() {
timeout -k 10 300 python -u -m pytest tests -m gpu -k "stage or profil or h48" -x -q --timeout 200 --timeout-method thread > gpurun_out/r06pe_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06pe_tests.txt
[ $rc -gt 1 ] && exit $rc
for i in 1 2; do
  timeout -k 10 200 python bench.py --config H48 --no-cpu --points= --fir-points= --steps 50 --from-dicts-steps 0 \
    --iso-steps 0 > gpurun_out/r06pe_h48_$i.json 2> gpurun_out/r06pe_h48_$i.log || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r06pe_h48_$i.json')); s=d['stage_ms']
print('H48', d['ms_per_step'], d['checked']['all_ok'], d.get('stage_sampling'), {k: s[k] for k in ('generate','spectral','fir_kernel','stereo','total','host_plan_wall')})"
done
timeout -k 10 200 python bench.py --no-cpu --points= --fir-points= --steps 40 --from-dicts-steps 0 --iso-steps 0 \
  > gpurun_out/r06pe_c3.json 2> gpurun_out/r06pe_c3.log || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/r06pe_c3.json')); s=d['stage_ms']
print('C3', d['ms_per_step'], d['checked']['all_ok'], d['roofline']['frac'], {k: s[k] for k in ('generate','spectral','overlap_add','fir_kernel','stereo','total')})"
}

# GPU box: H48 with stage events on every batch (1), every 4th, every 16th and
# none (0), alternating, same session.
prof_every_ab2() {
for i in 1 2; do
  for k in 1 4 16 0; do
    MSGPU_BENCH_PROFILE_EVERY=$k timeout -k 10 200 python bench.py --config H48 --no-cpu --points= --fir-points= \
      --steps 50 --from-dicts-steps 0 --iso-steps 0 > gpurun_out/r06pe2_${k}_$i.json 2> gpurun_out/r06pe2_${k}_$i.log || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r06pe2_${k}_$i.json'))
print('H48 every $k', $i, d['ms_per_step'], d['checked']['all_ok'])"
  done
done
}

# GPU box: H48 after 3 or 30 warmup steps, stage events every batch or none, alternating.
h48_warmup_ab() {
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
}

# GPU box: sub-batch sizes for C3 and C4 on the round-6 kernels (3 streams, default gate), alternating.
sub_sweep() {
run() {
  cfg=$1; sub=$2; i=$3
  timeout -k 10 200 python bench.py --config $cfg --no-cpu --points= --fir-points= --steps 30 --from-dicts-steps 0 \
    --iso-steps 0 --sub $sub > gpurun_out/r06ss_${cfg}_${sub}_$i.json 2> gpurun_out/r06ss_${cfg}_${sub}_$i.log || return $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r06ss_${cfg}_${sub}_$i.json'))
print('$cfg sub $sub', $i, d['ms_per_step'], d['checked']['all_ok'], d['config'].get('sub_batches_per_gpu'))"
}
for i in 1 2; do
  for sub in 342 256 205 171; do run C3 $sub $i || exit 1; done
  for sub in 171 128 256; do run C4 $sub $i || exit 1; done
done
}

# GPU box: k_spec3p (MSGPU_SPEC3P=1) against the two-event chain -- bits on the
# mixed batch and on C3 / C4, the spectral tests under the persistent form,
# then the isolated / timed A/B on C3 and C4.
s3p_check() {
L=audio-suite_amd/msgpu/libmsgpu.so
timeout -k 10 300 python tools/bits_ab.py "$L,MSGPU_SPEC3P=0" "$L,MSGPU_SPEC3P=1" > gpurun_out/r06u_bits.json 2> gpurun_out/r06u_bits.log
echo "bits rc=$?"; cat gpurun_out/r06u_bits.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_long_filters.py -k 'spec3_persistent or fir8_persistent' -m gpu -x -q -s --timeout 200 --timeout-method thread > gpurun_out/r06u_tests0.txt 2>&1; echo "persist test rc=$?"; tail -3 gpurun_out/r06u_tests0.txt
MSGPU_SPEC3P=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k 'spec3 or C3 or C4' -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06u_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06u_tests.txt
[ $rc -gt 1 ] && exit $rc
bash tools/ab_env.sh r06u 'p0|MSGPU_SPEC3P=0|base' 'p1|MSGPU_SPEC3P=1|base' 'p0b|MSGPU_SPEC3P=0|base' 'p1b|MSGPU_SPEC3P=1|base'
}

# GPU box: k_fir8p phase stamps against the number of persistent workgroups
# (MSGPU_FIR8P_CUS): does a block's segment-load phase shrink when fewer CUs
# share HBM (bandwidth share) or stay (latency)?
fir8_cus_stamps() {
for c in 256 128 64 16 8; do
  echo "=== $c workgroups"
  MSGPU_FIR8P_CUS=$c MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_firstamps.so timeout -k 10 200 python tools/fir8_stamps.py C3 256 || exit $?
done
}

# C3 with 2 / 3 / 4 streams (sub-batches of 512 / 342 / 256), default gate, alternating
c3_streams() {
for i in 1 2; do
  for cfg in "3 342" "2 512" "4 256"; do
    set -- $cfg
    timeout -k 10 200 python bench.py --no-cpu --points= --fir-points= --steps 30 --from-dicts-steps 0 --iso-steps 0 \
      --streams $1 --sub $2 > gpurun_out/r06c3s_$1_$i.json 2> gpurun_out/r06c3s_$1_$i.log || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r06c3s_$1_$i.json'))
print('C3 streams $1 sub $2', $i, d['ms_per_step'], d['checked']['all_ok'])"
  done
done
}

# C3 with 3 vs 2 streams, default gate, four alternating pairs
c3_streams32() {
for i in 1 2 3 4; do
  for cfg in "3 342" "2 512"; do
    set -- $cfg
    timeout -k 10 200 python bench.py --no-cpu --points= --fir-points= --steps 40 --from-dicts-steps 0 --iso-steps 0 \
      --streams $1 --sub $2 > gpurun_out/r06c32_$1_$i.json 2> gpurun_out/r06c32_$1_$i.log || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r06c32_$1_$i.json'))
print('C3 streams $1 sub $2', $i, d['ms_per_step'], d['checked']['all_ok'])"
  done
done
}

# FIR8 spectra with Ho at a 128-byte-aligned offset vs the HEAD library (libmsgpu_head.so): bits, FIR tests, C3 and FIR-point A/B
ho_check() {
timeout -k 10 300 python tools/bits_ab.py audio-suite_amd/msgpu/libmsgpu_head.so > gpurun_out/r06ho_bits.json 2>/dev/null; echo "bits rc=$?"; cat gpurun_out/r06ho_bits.json
timeout -k 10 400 python -u -m pytest tests/test_gpu_fir.py tests/test_gpu_long_filters.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06ho_tests.txt 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r06ho_tests.txt
[ $rc -gt 1 ] && exit $rc
bash tools/ab_env.sh r06ho "new|MSGPU_X=1|base" "old|MSGPU_X=1|head" "new2|MSGPU_X=1|base" "old2|MSGPU_X=1|head"
for lib in base head; do
  if [ $lib = base ]; then le=""; else le="MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_head.so"; fi
  env $le timeout -k 10 300 python bench.py --no-cpu --points= --steps 5 --from-dicts-steps 0 --iso-steps 0 > gpurun_out/r06ho_fir_$lib.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/r06ho_fir_$lib.json')); print('$lib', {k: (v['ms_per_step'], v['roofline']['frac'], v['check']['all_ok']) for k, v in d['points'].items()})"
done
}

# k_fir8q carry slot: nontemporal stores (nt1) / stores + loads (nt3) vs product, FIR points, alternating
q2nt_ab() {
L=$PWD/audio-suite_amd/msgpu
for rep in 1 2 3; do
  for lib in base nt1 nt3; do
    if [ $lib = base ]; then le=""; else le="MSGPU_LIB=$L/libmsgpu_$lib.so"; fi
    env $le timeout -k 10 300 python bench.py --no-cpu --points= --steps 5 --from-dicts-steps 0 --iso-steps 0 > gpurun_out/r06nt_$lib$rep.json 2>/dev/null || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r06nt_$lib$rep.json')); print('$lib$rep', {k: (v['ms_per_step'], v['roofline']['frac'], v['check']['all_ok']) for k, v in d['points'].items() if k.startswith('FIR')})"
  done
done
}

# maxbits zeroed through the batch upload (no fill launch): bits, stereo / peak tests, H48 and C3 A/B vs HEAD lib
mb_check() {
timeout -k 10 300 python tools/bits_ab.py audio-suite_amd/msgpu/libmsgpu_head.so > gpurun_out/r06mb_bits.json 2>/dev/null || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/r06mb_bits.json')); print('identical', d['identical'], d['differing_presets'])"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06mb_tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r06mb_tests.txt
[ $rc -ne 0 ] && exit $rc
bash tools/h48_ab.sh r06mb libmsgpu.so libmsgpu_head.so || exit $?
bash tools/ab_env.sh r06mb "new|MSGPU_X=1|base" "old|MSGPU_X=1|head" "new2|MSGPU_X=1|base" "old2|MSGPU_X=1|head"
}

# C5 sub-batch size: 171 (6 = 2 per stream, the default) vs 114 (9 = 3 per stream), alternating
c5_sub_ab() {
for i in ${C5_REPS:-1 2}; do
  for sub in ${C5_SUBS:-171 114}; do
    timeout -k 10 300 python bench.py --config C5 --no-cpu --points= --fir-points= --steps 3 --warmup 1 --iso-steps 0 \
      --from-dicts-steps 0 --sub $sub > gpurun_out/r06c5s_${sub}_$i.json 2> gpurun_out/r06c5s_${sub}_$i.log || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r06c5s_${sub}_$i.json'))
print('C5 sub $sub', $i, d['ms_per_step'], d['checked']['all_ok'], d['config'].get('sub_batches_per_gpu'), d['config'].get('stream_gate'))"
  done
done
}

# k_fir8q with the carry loaded one pair ahead (libmsgpu_a1.so, MSG_Q2_AHEAD=1) vs product, FIR points, alternating
q2_ahead1_ab() {
L=$PWD/audio-suite_amd/msgpu
for rep in 1 2 3; do
  for lib in base a1; do
    if [ $lib = base ]; then le=""; else le="MSGPU_LIB=$L/libmsgpu_$lib.so"; fi
    env $le timeout -k 10 300 python bench.py --no-cpu --points= --steps 5 --from-dicts-steps 0 --iso-steps 0 > gpurun_out/r06a1_$lib$rep.json 2>/dev/null || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r06a1_$lib$rep.json')); print('$lib$rep', {k: (v['ms_per_step'], v['roofline']['frac'], v['check']['all_ok']) for k, v in d['points'].items() if k.startswith('FIR')})"
  done
done
}

name=${1:?usage: tools/round6_ab.sh NAME [args]}; shift
"$name" "$@"
