#!/bin/bash
# GPU box: the new FIR edge test, smoke(), and bench.py under torch.distributed.run
# with one rank (the driver's multi-GPU launch path).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_fir.py -m gpu -v -s --timeout 200 --timeout-method thread \
  > gpurun_out/r03w_fir_tests.txt 2>&1 || { tail -30 gpurun_out/r03w_fir_tests.txt; exit 1; }
grep -E "rel rms|passed|failed" gpurun_out/r03w_fir_tests.txt | tail -14
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03w_smoke.txt 2>&1 || exit $?
cat gpurun_out/r03w_smoke.txt | tail -2
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 1 --steps 20 --warmup 3 --points= --no-cpu > gpurun_out/r03w_torchrun.json 2> gpurun_out/r03w_torchrun.log || exit $?
python3 -c "
import json; d=json.loads(open('gpurun_out/r03w_torchrun.json').read().strip().splitlines()[-1]); print('torchrun n_gpus', d['n_gpus'], 'step', d['ms_per_step'], 'value', d['value'], 'ranks', d['ranks'])"
