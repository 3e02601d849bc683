#!/bin/bash
# Round-end GPU job: all GPU tests, the bench line, its rocprofv3 kernel stats, the
# timing scripts, and a 2-rank rehearsal of the multi-GPU bench on one device.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash scripts/gpu_job.sh tests "tests" bench "--steps 20 --warmup 5" prof "--steps 20 --warmup 5" \
    script "scripts/filter_timing.py" script "scripts/util_diag.py" script "scripts/plan_prof.py" || exit $?
CASIM_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/multi2.json 2> gpurun_out/multi2.err || {
    echo "MULTI FAILED"; tail -20 gpurun_out/multi2.err; exit 1; }
cat gpurun_out/multi2.json
echo FINAL_OK
