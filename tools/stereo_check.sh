#!/bin/bash
# GPU box: a stereo-pass change against the kept library -- bits on the mixed
# batch, the stereo GPU tests, then C3 / C5 A/B (isolated stereo stage).
set -o pipefail
mkdir -p gpurun_out
tag=${1:?tag}; old=${2:?old lib name}
timeout -k 10 300 python tools/bits_ab.py audio-suite_amd/msgpu/$old > gpurun_out/${tag}_bits.json 2> gpurun_out/${tag}_bits.log
echo "bits rc=$?"; cat gpurun_out/${tag}_bits.json
timeout -k 10 400 python -u -m pytest tests -m gpu -k "stereo" -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${tag}_tests.txt
[ $rc -gt 1 ] && exit $rc
lib=${old#libmsgpu_}; lib=${lib%.so}
bash tools/ab_env.sh ${tag} "new|MSGPU_X=1|base" "old|MSGPU_X=1|$lib" "new2|MSGPU_X=1|base" "old2|MSGPU_X=1|$lib"
