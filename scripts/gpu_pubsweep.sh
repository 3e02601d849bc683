#!/bin/bash
# GPU-box job: Estimate parity tests (decoupled / publisher), then the publisher sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "publisher or decoupled or gosort or c2" > gpurun_out/pytest_pub.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_pub.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_pub.log; exit $rc; }
PUB_BLOCKS_LIST="64 128 256" PUB_CHUNK_LIST="16384 8192 4096" timeout -k 10 900 bash scripts/pub_sweep.sh
echo PUBSWEEP_OK
