#!/bin/bash
# (variant builds: make -C autoscaler_amd/csrc OUT=../lib/<name> BUILD=../../build/<name> "EXTRA=-DCASIM_PC_SKY=.. -DCASIM_PC_BULK_FAILS=.. -DCASIM_PC_BULK_SKIP=.. / -DCASIM_FB_BACKOFF=.. / -DCASIM_FB_ROWWISE_MAX=..")
# GPU-box job: FilterOutSchedulable A/B over several builds (the bitmap walk's back-off and
# row-wise update threshold: autoscaler_amd/lib/fb{1,2,4,8}), alternating processes
# on C5 and C5-loose; every run must report parity with the CPU port.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ab_fb2.txt
for r in 0 1 2; do
  for lib in autoscaler_amd/lib/libcasim.so autoscaler_amd/lib/fb1/libcasim.so autoscaler_amd/lib/fb2/libcasim.so \
             autoscaler_amd/lib/fb4/libcasim.so autoscaler_amd/lib/fb8/libcasim.so; do
    CASIM_LIB_PATH=$PWD/$lib timeout -k 10 200 python -u scripts/filter_timing.py c5 c5-loose > gpurun_out/ab_one.txt 2>&1 \
      || { tail -20 gpurun_out/ab_one.txt; exit 1; }
    sed "s|^|$r $lib |; s/ evals=.*call_ms/ call_ms/" gpurun_out/ab_one.txt | cut -c1-150 >> gpurun_out/ab_fb2.txt
  done
done
cat gpurun_out/ab_fb2.txt
! grep -q "parity=False" gpurun_out/ab_fb2.txt
