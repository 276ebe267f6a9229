set -o pipefail
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
