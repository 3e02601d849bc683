#!/bin/bash
# GPU-box job: publisher block / chunk A/B, configurations interleaved and repeated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
H="--no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util --no-filter --no-unlimited --no-runonce --no-planner"
for rep in 1 2 3; do
  for cfg in "128 8192" "64 16384" "128 16384" "64 8192" "192 8192"; do
    set -- $cfg
    r=$(CASIM_KNOBS=1 CASIM_PUB_BLOCKS=$1 CASIM_PUB_CHUNK=$2 timeout -k 10 120 python bench.py $H --steps 30 --warmup 3 2>/dev/null \
        | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);e=d['extra'];print(round(d['ms_per_step'],4), round(e['device_resident']['ms_per_step'],4))") || exit 1
    echo "rep=$rep blocks=$1 chunk=$2 headline_ms device_ms: $r"
  done
done
echo PUBSWEEP2_OK
