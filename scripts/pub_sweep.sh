#!/bin/bash
# Publisher tuning sweep: C2 step time for publisher block counts and chunk sizes.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for pb in 16 32 64 128; do
  for ch in 4096 16384; do
    r=$(CASIM_PUB_BLOCKS=$pb CASIM_PUB_CHUNK=$ch timeout -k 10 120 python bench.py --no-sweep --no-c4 --no-cpu-baseline --steps 10 2>/dev/null \
        | python3 -c "import json,sys;d=json.load(sys.stdin);print(round(d['ms_per_step'],4), round(d['extra']['phases_ms']['chain_ms'],4))") || exit 1
    echo "blocks=$pb chunk=$ch ms_per_step/chain: $r"
  done
done
