#!/bin/bash
# diagnostics: fused stereo under 1 and 3 streams, each step bounded
mkdir -p gpurun_out
T=${1:-r05b}
run() { tag=$1; shift; echo "=== $tag $(date +%T)"; timeout -k 5 100 "$@" > gpurun_out/${T}_$tag.json 2> gpurun_out/${T}_$tag.log; rc=$?; echo "rc=$rc"; python3 tools/brief.py gpurun_out/${T}_$tag.json; return $rc; }
run s3 python bench.py --no-cpu --points '' --steps 20 --iso-steps 2 --from-dicts-steps 0 || exit 0
MSGPU_STEREO_FUSED=0 run s3off python bench.py --no-cpu --points '' --steps 20 --iso-steps 2 --from-dicts-steps 0 || exit 0
run s3b python bench.py --no-cpu --points '' --steps 20 --iso-steps 2 --from-dicts-steps 0 || exit 0
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/${T}_gpu_tests.txt
