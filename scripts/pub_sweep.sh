#!/bin/bash
# Publisher tuning sweep: C2 step time (device-resident and PCIe-inclusive) for publisher
# block counts and chunk sizes.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for pb in ${PUB_BLOCKS_LIST:-16 32 64 128}; do
  for ch in ${PUB_CHUNK_LIST:-4096 16384}; do
    r=$(CASIM_PUB_BLOCKS=$pb CASIM_PUB_CHUNK=$ch timeout -k 10 120 python bench.py --no-sweep --no-c4 --no-cpu-baseline --steps 20 2>/dev/null \
        | python3 -c "import json,sys;d=json.load(sys.stdin);print(round(d['ms_per_step'],4), round(d['extra']['phases_ms']['chain_ms'],4), round(d['extra']['pcie_inclusive']['ms_per_step'],4))") || exit 1
    echo "blocks=$pb chunk=$ch device_ms chain_ms pcie_ms: $r"
  done
done
