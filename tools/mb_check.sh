# maxbits zeroed through the batch upload (no fill launch): bits, stereo / peak tests, H48 and C3 A/B vs HEAD lib
set -o pipefail
timeout -k 10 300 python tools/bits_ab.py audio-suite_amd/msgpu/libmsgpu_head.so > gpurun_out/r06mb_bits.json 2>/dev/null || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/r06mb_bits.json')); print('identical', d['identical'], d['differing_presets'])"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06mb_tests.txt 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r06mb_tests.txt
[ $rc -ne 0 ] && exit $rc
bash tools/h48_ab.sh r06mb libmsgpu.so libmsgpu_head.so || exit $?
bash tools/ab_env.sh r06mb "new|MSGPU_X=1|base" "old|MSGPU_X=1|head" "new2|MSGPU_X=1|base" "old2|MSGPU_X=1|head"
