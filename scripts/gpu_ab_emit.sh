#!/bin/bash
# GPU-box job: headline A/B — run-head emission inside k_run_table (default) against the
# separate k_emit_runs launch (CASIM_EMIT_SEPARATE=1), and a kernel trace of the latter
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
H="--no-cpu-baseline --no-sweep --no-c4 --no-expansion --no-util --no-filter --no-unlimited --no-runonce --no-planner"
summ() { python3 -c "
import json,sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e = d['extra']
print(sys.argv[2], 'headline', round(d['ms_per_step'], 4), 'device', round(e['device_resident']['ms_per_step'], 4), 'i32', round(e['host_int32_ids']['ms_per_step'], 4))
" "$1" "$2"; }
for rep in 1 2; do
timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 $H > gpurun_out/ab_fused.json 2> gpurun_out/ab_fused.err || { tail gpurun_out/ab_fused.err; exit 1; }
summ gpurun_out/ab_fused.json fused
CASIM_EMIT_SEPARATE=1 timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 $H > gpurun_out/ab_sep.json 2> gpurun_out/ab_sep.err || { tail gpurun_out/ab_sep.err; exit 1; }
summ gpurun_out/ab_sep.json separate
done
export TMPDIR=/tmp
cd /tmp && CASIM_EMIT_SEPARATE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/tl_sep" -o run --output-format csv -- \
   python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 2 $H > "$GRAFT_REPO_ROOT/gpurun_out/tl_sep.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/tl_sep.log"; exit 1; }
cd "$GRAFT_REPO_ROOT"
f=$(find gpurun_out/tl_sep -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_timeline.py "$f" > gpurun_out/tl_sep.txt
echo AB_EMIT_OK
