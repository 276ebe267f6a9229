#!/bin/bash
# k_er_gains v2 (per-tap runs + slot sums): suite, then kernel stats of a C4 bench (its launch time under rocprofv3)
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q -s --timeout 250 --timeout-method thread \
  > gpurun_out/r05ao_gpu_tests.txt 2>&1; rc=$?; echo "suite rc=$rc"; grep -E "FAILED|passed|failed|host-drawn" gpurun_out/r05ao_gpu_tests.txt | tail -6
if [ $rc -ne 0 ]; then exit $rc; fi
R=$PWD; export TMPDIR=/tmp; cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r05ao_C4" -o run -- \
  python3 "$R/bench.py" --config C4 --no-cpu --iso-steps 0 --points= --steps 10 > "$R/gpurun_out/r05ao_C4_bench.json" 2> "$R/gpurun_out/r05ao_C4.log" || exit $?
cd "$R"; grep -h "k_er_gains\|k_fir8_hconv" gpurun_out/r05ao_C4/*kernel_stats.csv | cut -c1-160
