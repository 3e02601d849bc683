#!/bin/bash
# C4 Estimate with and without the heavy-first split (device-resident results).
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for v in "" 1; do
  r=$(CASIM_KNOBS=1 CASIM_NO_SPLIT=$v timeout -k 10 180 python bench.py --no-sweep --no-cpu-baseline --steps 10 2>/dev/null \
      | python3 -c "import json,sys;d=json.load(sys.stdin);print(round(d['ms_per_step'],4), round(d['extra']['c4']['estimate_ms'],4))") || exit 1
  echo "no_split=${v:-0} c2_ms c4_ms: $r"
done
