#!/bin/bash
# GPU-box job (round 5): N = 2 rehearsal of bench.py's weak-scaling path on the one GPU
# (two ranks share the card; gloo collectives), as the driver launches N > 1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CASIM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
   --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 \
   > gpurun_out/multi2.json 2> gpurun_out/multi2.err || { echo MULTI FAILED; tail -30 gpurun_out/multi2.err; exit 1; }
tail -c 1500 gpurun_out/multi2.json
echo N2_OK
