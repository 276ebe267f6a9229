#!/bin/bash
# GPU box (one GPU): rehearse the multi-rank / multi-worker paths with every
# rank on device 0 -- the library's DevicePool (2 workers), then bench.py with
# 2 ranks under torch.distributed.run (the driver's launch form) and under its
# own --gpus launcher.  Not scaling points: the ranks share one GPU.
set -o pipefail
tag=${1:?usage: tools/multi_round.sh TAG}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/multi_rehearsal.py 2 > gpurun_out/${tag}_pool.json 2> gpurun_out/${tag}_pool.log || exit $?
cat gpurun_out/${tag}_pool.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu --points= --fir-points= --iso-steps 0 \
  --from-dicts-steps 0 --rehearse-one-gpu > gpurun_out/${tag}_tdr.json 2> gpurun_out/${tag}_tdr.log || exit $?
timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu --points= --fir-points= --iso-steps 0 \
  --from-dicts-steps 0 --rehearse-one-gpu > gpurun_out/${tag}_self.json 2> gpurun_out/${tag}_self.log || exit $?
python3 - gpurun_out/${tag}_tdr.json gpurun_out/${tag}_self.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    print(f, "n_gpus", d["n_gpus"], "ms/step", d["ms_per_step"], "value", d["value"], "ok", d["checked"]["all_ok"],
          "ranks", [(r["rank"], r["device"], r["seeds"], r["elapsed_s"]) for r in d["ranks"]], d["config"]["parallelism"])
PY
