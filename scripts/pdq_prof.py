"""Phase cycle counters of the device Go sort (CASIM_PROF build: make -C autoscaler_amd/csrc
prof) on the rank sequences of the heaviest C2 groups (scripts/gpu_job.sh script ...)."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("CASIM_LIB_PATH", os.path.join(ROOT, "autoscaler_amd", "lib", "libcasim_prof.so"))
from autoscaler_amd import native, workloads as W  # noqa: E402

lib = native.load()
lib.ca_debug_pdq_prof.argtypes = [C.c_void_p, C.c_int32]
NAMES = ["total", "init", "pop", "phaseA", "plist", "partition", "P2", "P3", "-", "D", "small",
         "steps", "frames", "part_frames", "small_frames", "elems_partitioned"]
w = W.c2()
p = w.table.pods
sizes = np.diff(w.group_off)
for g in np.argsort(-sizes)[:3]:
    idx = w.pod_idx[w.group_off[g]:w.group_off[g + 1]]
    ac = float(w.templates[g]["node"]["alloc_milli_cpu"]); am = float(w.templates[g]["node"]["alloc_memory"])
    score = p["score_milli_cpu"][idx] / ac + p["score_memory"][idx] / am
    ranks = np.unique(-score, return_inverse=True)[1].astype(np.uint32)
    for store in (1, 2):
        out = np.zeros(32 + 256 + 8 + 384, np.uint64)
        native.go_sort_ranks(ranks, store=store)
        lib.ca_debug_pdq_prof(out.ctypes.data, 1)
        t0 = time.perf_counter()
        native.go_sort_ranks(ranks, store=store)
        dt = time.perf_counter() - t0
        lib.ca_debug_pdq_prof(out.ctypes.data, 1)
        print(f"group {g} n={len(ranks)} store={store} call {dt*1e3:.3f} ms")
        print("   " + "  ".join(f"{n}={int(v)}" for n, v in zip(NAMES, out[:16]) if n != "-"))
        print("   phaseA sums over waves: breakPatterns=%d choosePivot=%d reverse=%d pis=%d pis_calls(w0)=%d"
              % tuple(int(x) for x in out[16:21]))
        print("   pis (wave 0): descent=%d land=%d shift=%d moved=%d len_sum=%d steps=%d"
              % tuple(int(x) for x in out[21:27]))
        print("   P3 waves: cycles_sum=%d iters_sum=%d iters_max=%d"
              % tuple(int(x) for x in out[27:30]))
        pz = out[288:296].astype(np.int64)
        print("   wave pis (all waves): find_cyc=%d rot_cyc=%d search_trips=%d rot_trips=%d steps=%d calls=%d quads=%d"
              % tuple(int(x) for x in pz[:7]))
        if pz[2] > 0 and pz[3] > 0:
            print("   per search trip %.0f cyc, per rotate trip %.0f cyc" % (pz[0] / pz[2], pz[1] / pz[3]))
        print("   step   nf   np   A1wall A1maxw  wgpis(n)      A2  plist      P1      P2      P3       D  elems  wpis_max cp_max wpis_len")
        for st in range(16):
            r = out[32 + 16 * st: 48 + 16 * st].astype(np.int64)
            if r[0] == 0:
                continue
            print("   %4d %4d %4d %8d %6d %8d(%d) %7d %6d %7d %7d %7d %7d %6d %9d %6d %8d" % (
                st, r[0], r[1], r[2], r[11], r[3], r[12], r[4], r[5], r[6], r[7], r[8], r[9], r[10], r[13], r[14], r[15]))

# every group's sort in the headline configuration (the C2 plan, decoupled Go order):
# per-workgroup kernel / prologue / epilogue cycles
m = native.Mirror(0)
W.load_estimate(m, w)
plan = native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates)
plan.set_phase_timing(False)
for _ in range(3):
    plan.run_u16(w.max_nodes, 0, copy=False)
out = np.zeros(32 + 256 + 8 + 384, np.uint64)
lib.ca_debug_pdq_prof(out.ctypes.data, 1)
plan.run_u16(w.max_nodes, 0, copy=False)
out[:] = 0
lib.ca_debug_pdq_prof(out.ctypes.data, 0)
wg = out[296:296 + 384].reshape(128, 3).astype(np.int64)[: len(w.templates)]
order = np.argsort(-wg[:, 0])
print("plan sorts: kernel cycles max %d median %d min %d" % (wg[:, 0].max(), np.median(wg[:, 0]), wg[:, 0].min()))
for g in order[:8]:
    print("   group %3d n=%d: total %d prologue %d epilogue %d" % (g, sizes[g], wg[g, 0], wg[g, 1], wg[g, 2]))
