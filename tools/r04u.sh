#!/bin/bash
# GPU box: bit-identity test of the persistent FIR, then the C3 / C4 schedule
# re-swept with it (streams x gate).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_long_filters.py -m gpu -q -x --timeout 200 \
  --timeout-method thread -k "fir8 or fir64" > gpurun_out/r04u_tests.txt 2>&1 || { tail -20 gpurun_out/r04u_tests.txt; exit 1; }
tail -1 gpurun_out/r04u_tests.txt
run() {  # tag, args...
  local t=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu --iso-steps 0 --from-dicts-steps 0 --points= "$@" > gpurun_out/r04u_$t.json 2> gpurun_out/r04u_$t.log || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r04u_$t.json')); print('$t', d['ms_per_step'], d['checked']['all_ok'])"
}
run C3_s3g24 --config C3 --steps 30
run C3_s3u --config C3 --steps 30 --gate none
run C3_s2g24 --config C3 --steps 30 --streams 2
run C3_s4g24 --config C3 --steps 30 --streams 4
run C3_s3g23 --config C3 --steps 30 --gate 2,3
run C3_s3g24b --config C3 --steps 30
run C4_s3g24 --config C4 --steps 30
run C4_s3u --config C4 --steps 30 --gate none
run C4_s2g24 --config C4 --steps 30 --streams 2
