"""Phase profile of the device-chain planner (ca_plan_removals, plan_chain.hip) on C3 at the
bench's limits: host timings and the kernel's shader-clock counters per phase.
(scripts/gpu_job.sh script "scripts/plan_prof.py [n_nodes]")"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("CASIM_LIB_PATH", os.path.join(ROOT, "autoscaler_amd", "lib", "libcasim_prof.so")) if "--prof" in sys.argv else None
sys.argv = [a for a in sys.argv if a != "--prof"]
os.environ["CASIM_KNOBS"] = "1"          # CASIM_PLAN_HELPERS is a knob (read only with CASIM_KNOBS)
from autoscaler_amd import native, workloads as W  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
w = W.c3(n_nodes=n)
args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
hints = np.full(len(w.table), -1, np.int32)
helpers = os.environ.get("CASIM_PLAN_HELPERS", "7")
print(f"helper waves: {helpers}")
for limit in (20, 200, 0):
    m = native.Mirror(0)
    W.load_sweep(m, w)
    for rep in range(3):
        m.fork()
        t = time.perf_counter()
        r = m.plan_removals(*args, hints, 0, limit)
        dt = (time.perf_counter() - t) * 1e3
        st = m.plan_stats()
        pr = m.plan_chain_profile()
        m.revert()
    tot = max(pr.get("total", 1), 1)
    ghz = tot / (pr["kernel_ms"] * 1e6) if pr["kernel_ms"] > 0 else 0
    print(f"limit {limit}: {dt:.3f} ms (library {st['total_ms']:.3f}) path {st['path']} simulated {st['simulated']} "
          f"evals {int(r.results['evals'].sum())} moves {len(r.moves)}", flush=True)
    print("   host: " + "  ".join(f"{k}={pr[k]:.3f}" for k in
                                   ("sync_ms", "launch_kernel_ms", "kernel_ms", "readback_ms", "replay_ms")))
    print(f"   kernel clock {ghz:.2f} GHz; phases (% of total cycles): " +
          "  ".join(f"{k}={100 * pr[k] / tot:.1f}" for k in
                    ("init", "lists", "pdb", "fork", "bulk", "prep", "hint", "win", "loadchk", "skyb", "scan", "add",
                     "commit", "revert")))
    print(f"   blocks scanned {pr['blocks']}  skip windows {pr['windows']}  helper hand-offs {pr.get('handoffs', 0)}",
          flush=True)
    if pr.get("r_npods"):
        print("   plain runs: {r_nruns} runs, pods {r_npods} blocks {r_nblk} windows {r_nwin} sky rebuilds {r_nsky}; cycles/pod: pod {a:.0f} win {b:.0f} blk {c:.0f} "
              "sky {d:.0f} add {e:.0f}".format(a=pr["r_pod"] / pr["r_npods"], b=pr["r_win"] / pr["r_npods"],
                                              c=pr["r_blk"] / pr["r_npods"], d=pr["r_sky"] / pr["r_npods"],
                                              e=pr["r_add"] / pr["r_npods"], **pr), flush=True)
    t = time.perf_counter()
    native.plan_args(*args, hints)
    print(f"   plan_args (the wrapper's marshalling) {(time.perf_counter() - t) * 1e3:.3f} ms", flush=True)
    m.close()
