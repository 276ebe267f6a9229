# k_fir8q carry slot: nontemporal stores (nt1) / stores + loads (nt3) vs product, FIR points, alternating
set -o pipefail
L=$PWD/audio-suite_amd/msgpu
for rep in 1 2 3; do
  for lib in base nt1 nt3; do
    if [ $lib = base ]; then le=""; else le="MSGPU_LIB=$L/libmsgpu_$lib.so"; fi
    env $le timeout -k 10 300 python bench.py --no-cpu --points= --steps 5 --from-dicts-steps 0 --iso-steps 0 > gpurun_out/r06nt_$lib$rep.json 2>/dev/null || exit $?
    python3 -c "
import json; d=json.load(open('gpurun_out/r06nt_$lib$rep.json')); print('$lib$rep', {k: (v['ms_per_step'], v['roofline']['frac'], v['check']['all_ok']) for k, v in d['points'].items() if k.startswith('FIR')})"
  done
done
