#!/bin/bash
# GPU-box job: FilterOutSchedulable A/B of the default build (autoscaler_amd/lib/libcasim.so)
# against a baseline build (autoscaler_amd/lib/ab/), alternating processes on C5 and C5-loose.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ab_replay.txt
for r in 0 1 2 3; do
  for lib in autoscaler_amd/lib/ab/libcasim.so autoscaler_amd/lib/libcasim.so; do
    CASIM_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u scripts/filter_timing.py c5 c5-loose > gpurun_out/ab_one.txt 2>&1 \
      || { tail -20 gpurun_out/ab_one.txt; exit 1; }
    sed "s|^|$r $lib |; s/ evals=.*call_ms/ call_ms/" gpurun_out/ab_one.txt | cut -c1-150 >> gpurun_out/ab_replay.txt
  done
done
cat gpurun_out/ab_replay.txt
