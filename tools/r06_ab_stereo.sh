set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/bits_ab.py audio-suite_amd/msgpu/libmsgpu_r05.so > gpurun_out/r06d_bits.json 2> gpurun_out/r06d_bits.log; echo "bits rc=$?"; cat gpurun_out/r06d_bits.json
timeout -k 10 400 bash tools/lib_ab.sh r05 base r05 base 2>&1 | tee gpurun_out/r06d_ab.txt || exit 1
for v in r05 base; do
  if [ $v != base ]; then export MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_$v.so; else unset MSGPU_LIB; fi
  timeout -k 10 200 python bench.py --config C5 --no-cpu --points= --fir-points= --steps 5 > gpurun_out/r06d_c5_$v.json 2>/dev/null || exit 1
  python3 -c "
import json;d=json.load(open('gpurun_out/r06d_c5_$v.json'));i=d['roofline_isolated']['stage_ms'];t=d['stage_ms']
print('C5 $v', 'step', d['ms_per_step'], 'ok', d['checked']['all_ok'], 'iso stereo', i['stereo'], 'timed stereo', t['stereo'])" | tee -a gpurun_out/r06d_ab.txt
done
