"""A/B of two builds of the library on the bench's headline step (C2, results on the host
as 16-bit podset indices, phase events off): alternating processes, each timing 40 steps
after warmup.  Usage: python scripts/ab_lib.py LIB_A LIB_B [LIB ...] [rounds]"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import os, sys, time
sys.path.insert(0, %r)
from autoscaler_amd import native, workloads as W
w = W.c2()
m = native.Mirror(0)
W.load_estimate(m, w)
with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
    plan.set_phase_timing(False)
    for _ in range(5):
        plan.run_u16(w.max_nodes, 0, copy=False)
    ts = []
    for _ in range(40):
        t = time.perf_counter()
        plan.run_u16(w.max_nodes, 0, copy=False)
        ts.append((time.perf_counter() - t) * 1e3)
    ts.sort()
    print(ts[len(ts) // 2], ts[0])
""" % ROOT

args = sys.argv[1:]
rounds = int(args.pop()) if args and args[-1].isdigit() else 3
libs = args
res = {lib: [] for lib in libs}
for r in range(rounds):
    for lib in libs:
        env = dict(os.environ, CASIM_LIB_PATH=os.path.abspath(lib))
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(out.stderr[-2000:])
            sys.exit(1)
        med, mn = map(float, out.stdout.split())
        res[lib].append(med)
        print(f"round {r} {os.path.basename(os.path.dirname(lib)) or lib}/{os.path.basename(lib)}: median {med:.4f} min {mn:.4f}", flush=True)
for lib, v in res.items():
    print(f"{lib}: median of medians {np.median(v):.4f} ms ({', '.join(f'{x:.4f}' for x in v)})")
