#!/bin/bash
# GPU box: fir64 route tests, then C4 / C5 schedule sweeps (streams x gate) and
# the SQ counters of the C5 kernels on one stream.
set -o pipefail
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_long_filters.py -m gpu -q -x --timeout 200 --timeout-method thread \
  -k "fir64 or long_space" > gpurun_out/r04m_tests.txt 2>&1 || exit $?
tail -2 gpurun_out/r04m_tests.txt
run() {  # tag, args...
  local t=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu --iso-steps 0 --from-dicts-steps 0 --points= "$@" > gpurun_out/r04m_$t.json 2> gpurun_out/r04m_$t.log || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/r04m_$t.json')); print('$t', d['ms_per_step'], d['checked']['all_ok'])"
}
run C4_s3g24 --config C4 --steps 30
run C4_s3u --config C4 --steps 30 --gate none
run C4_s2g24 --config C4 --steps 30 --streams 2
run C5_s3u --config C5 --steps 3 --gate none
run C5_s2u --config C5 --steps 3 --gate none --streams 2
run C5_s1 --config C5 --steps 3 --gate none --streams 1
run C5_s3g24 --config C5 --steps 3
cd /tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    --output-format csv -d "$R/gpurun_out/r04m_C5_sq" -o run -- \
    python3 "$R/bench.py" --config C5 --steps 1 --warmup 1 --no-cpu --iso-steps 0 --from-dicts-steps 0 --points= --streams 1 --gate none \
    > "$R/gpurun_out/r04m_C5_sq.log" 2>&1 || exit $?
cd "$R"
python3 tools/pmc_summary.py gpurun_out/r04m_C5_sq > gpurun_out/r04m_C5_sq_summary.txt 2>&1 || true
grep -E "^k_|^void|VALU/WAVE|WAIT_ANY/" gpurun_out/r04m_C5_sq_summary.txt | head -60
