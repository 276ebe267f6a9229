for n in prod 16; do
  if [ $n = prod ]; then L=""; else L="MSGPU_LIB=$PWD/audio-suite_amd/msgpu/libmsgpu_$n.so"; fi
  env $L timeout -k 10 150 python -u bench.py --no-cpu --points= --steps 5 > gpurun_out/gv_$n.json 2>/dev/null || exit 3
done
