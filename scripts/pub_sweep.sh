#!/bin/bash
# Publisher tuning sweep: C2 headline step (results on the host) and chain time for
# publisher block counts and chunk sizes.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
H="--no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util --no-filter --no-unlimited --no-runonce --no-planner"
for pb in ${PUB_BLOCKS_LIST:-8 16 32 64}; do
  for ch in ${PUB_CHUNK_LIST:-2048 4096 8192}; do
    r=$(CASIM_KNOBS=1 CASIM_PUB_BLOCKS=$pb CASIM_PUB_CHUNK=$ch timeout -k 10 120 python bench.py $H --steps 20 --warmup 3 2>/dev/null \
        | python3 -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);e=d['extra'];print(round(d['ms_per_step'],4), round(e['phases_ms']['chain_ms'],4), round(e['host_int32_ids']['ms_per_step'],4))") || exit 1
    echo "blocks=$pb chunk=$ch headline_ms chain_ms int32_ms: $r"
  done
done
