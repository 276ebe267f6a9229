#!/bin/bash
# GPU box: a quick check after a kernel change -- the named test files (-m gpu),
# the bit A/B against a kept library build (tools/bits_ab.py) when one is named,
# and a short bench (headline + the standalone FIR points, no CPU baseline).
#   usage (on the box): bash tools/gpu_quick.sh TAG "tests/a.py tests/b.py" [libmsgpu_<old>.so]
set -o pipefail
tag=${1:?tag}; tests=${2:-tests}; old=$3
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest $tests -m gpu -v -s --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_tests.txt 2>&1
rc=$?
echo "== tests rc=$rc"; grep -E "FAILED|passed|failed|rel rms" gpurun_out/${tag}_tests.txt | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
if [ -n "$old" ]; then
  timeout -k 10 300 python tools/bits_ab.py audio-suite_amd/msgpu/$old > gpurun_out/${tag}_bits.json 2> gpurun_out/${tag}_bits.log
  echo "== bits rc=$?"; cat gpurun_out/${tag}_bits.json
fi
timeout -k 10 300 python bench.py --no-cpu --points= --steps 10 --from-dicts-steps 0 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.log || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/${tag}_bench.json'))
print('C3', d['ms_per_step'], d['checked']['all_ok'], 'iso', {k: d['roofline_isolated']['stage_ms'][k] for k in ('generate','spectral','overlap_add','fir_kernel','fir_h','stereo')})
print(json.dumps(d['points_summary']))
for k, v in d['points'].items(): print(k, v.get('fir_shape'), v['roofline']['kernel_ms'], v['roofline']['frac'], v['check']['all_ok'])"
