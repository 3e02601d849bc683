"""FilterOutSchedulable timing: ca_filter_out_schedulable vs the CPU port on C5-filter
variants, with the kernel's batch/cut counters (python scripts/filter_timing.py)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

from autoscaler_amd import native, workloads as W  # noqa: E402
import pyoracle  # noqa: E402

CFGS = {
    "c5": dict(),
    "c5-c4": dict(taints=True),
    "c5-nohints": dict(hint_frac=0.0),
    "c5-allhints": dict(hint_frac=1.0),
    "c5-loose": dict(util_low=(0.2, 0.4), util_high=(0.5, 0.7)),
    "c5-loose-nohints": dict(util_low=(0.2, 0.4), util_high=(0.5, 0.7), hint_frac=0.0),
    "c5-loose-allhints": dict(util_low=(0.2, 0.4), util_high=(0.5, 0.7), hint_frac=1.0),
}
args = sys.argv[1:]
if "--prof" in args:                    # CASIM_PROF build: the walk's cycle counters
    args.remove("--prof")
    os.environ["CASIM_LIB_PATH"] = os.path.join(ROOT, "autoscaler_amd", "lib", "libcasim_prof.so")
if "--bulk" in args:                    # (with --prof) fbcyc = mixed runs' chain / row loads / updates
    args.remove("--bulk")
    os.environ["CASIM_FB_PROF_BULK"] = "1"
    os.environ["CASIM_KNOBS"] = "1"
if "--phases" in args:                  # host phase marks of every call on stderr (filter.hip tmark)
    args.remove("--phases")
    os.environ["CASIM_DEBUG_TIMING"] = "1"
    os.environ["CASIM_KNOBS"] = "1"
names = args or list(CFGS)
for name in names:
    w = W.c5_filter(**CFGS[name])
    g, o = native.Mirror(0), pyoracle.OracleState()
    W.load_filter(g, w)
    W.load_filter(o, w)
    ts, ks = [], []
    for rep in range(4):
        g.fork()
        t = time.perf_counter()
        rg = g.filter_out_schedulable(w.pending, w.order, w.class_owner, w.hints, 0)
        ts.append((time.perf_counter() - t) * 1e3)
        st = g.filter_stats()
        ks.append(st["kernel_ms"])
        g.revert()
    o.fork()
    t = time.perf_counter()
    ro = o.filter_out_schedulable(w.pending, w.order, w.class_owner, w.hints, 0)
    cpu = (time.perf_counter() - t) * 1e3
    ok = np.array_equal(rg.node, ro.node) and rg.evals == ro.evals and rg.last_index == ro.last_index
    print(f"{name:12s} parity={ok} placed={rg.placed}/{len(w.order)} evals={rg.evals} call_ms={np.median(ts):.2f} "
          f"kernel_ms={np.median(ks):.2f} steps={st['block_steps']} rings={st['ring_scans']} "
          f"windows={st['windows']} seq_share={st['seq_share']:.2f} walk_cyc/pod={st['walk_cycles_per_pod']:.0f} "
          f"path={st['path']} S={st['shapes']} K={st['static_classes']} "
          f"statlds={st['static_in_lds']} fbcyc={[round(x) for x in st['fb_cycles_per_pod']]} cpu_ms={cpu:.1f} "
          f"x{cpu / np.median(ts):.1f}", flush=True)
    g.close()
