"""A/B of library builds on the C3 sweep (FindNodesToRemove over 5k nodes / 150k pods,
resident removal plan, bench.py's sweep leg): alternating processes, each timing 'fresh'
and 'hinted' loops (median of 15 after 3 warm-ups) and printing a digest of the results and
hints, which must agree across builds.  Usage: python scripts/ab_sweep.py LIB [LIB ...] [rounds]"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import hashlib, json, sys, time
sys.path.insert(0, %r)
import numpy as np
from autoscaler_amd import native, workloads as W
w = W.c3(n_nodes=5000)
m = native.Mirror(0)
W.load_sweep(m, w)
args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
fresh = np.full(len(w.table), -1, np.int32)
out = {}
with native.RemovalPlan(m, *args) as plan:
    for mode in ("fresh", "hinted"):
        ts = []
        for it in range(18):
            if mode == "fresh":
                m.set_hints(fresh)
            t = time.perf_counter()
            r = plan.run(0)
            if it >= 3:
                ts.append((time.perf_counter() - t) * 1e3)
        h = m.get_hints(len(w.table))
        dig = hashlib.sha1(np.ascontiguousarray(r.results).tobytes() + np.ascontiguousarray(h).tobytes()).hexdigest()[:12]
        out[mode] = [float(np.median(ts)), dig]
print(json.dumps(out))
""" % ROOT

args = sys.argv[1:]
rounds = int(args.pop()) if args and args[-1].isdigit() else 3
libs = args
res = {lib: [] for lib in libs}
digs = set()
for r in range(rounds):
    for lib in libs:
        env = dict(os.environ, CASIM_LIB_PATH=os.path.abspath(lib))
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        if out.returncode != 0:
            print(out.stderr[-2000:])
            sys.exit(1)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        res[lib].append(d)
        digs.add(tuple(v[1] for v in d.values()))
        print(f"round {r} {lib}: " + " ".join(f"{k} {v[0]:.4f} ms [{v[1]}]" for k, v in d.items()), flush=True)
for lib, v in res.items():
    print(f"{lib}: median " + " ".join(f"{k} {np.median([x[k][0] for x in v]):.4f} ms" for k in v[0]))
print("digests agree" if len(digs) == 1 else f"DIGESTS DIFFER: {digs}")
sys.exit(0 if len(digs) == 1 else 3)
