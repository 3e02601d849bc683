"""A/B of library builds on the planner loop (ca_plan_removals, C3 5k nodes / 150k pods,
candidates = all nodes): alternating processes, each timing limits 200 and none (median of
5 warm calls inside reverted forks) and printing a digest of the moves and results, which
must agree across builds.  Usage: python scripts/ab_planner.py LIB [LIB ...] [--rounds R]"""
import hashlib
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
args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
m = native.Mirror(0)
W.load_sweep(m, w)
out = {}
for limit in (200, 0):
    ts, dig = [], None
    for rep in range(6):
        hints = np.full(len(w.table), -1, np.int32)
        m.fork()
        t = time.perf_counter()
        r = m.plan_removals(*args, hints, 0, limit)
        ts.append((time.perf_counter() - t) * 1e3)
        h = hashlib.sha1(np.ascontiguousarray(r.moves).tobytes() + np.ascontiguousarray(r.results).tobytes() + hints.tobytes())
        dig = h.hexdigest()[:12]
        m.revert()
    out[str(limit)] = [float(np.median(ts[1:])), dig]
print(json.dumps(out))
""" % ROOT

argv = sys.argv[1:]
rounds = 3
if "--rounds" in argv:
    i = argv.index("--rounds")
    rounds = int(argv[i + 1])
    del argv[i:i + 2]
libs = argv
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
        print(f"round {r} {lib}: " + " ".join(f"limit {k} {v[0]:.3f} ms [{v[1]}]" for k, v in d.items()), flush=True)
for lib, v in res.items():
    print(f"{lib}: median " + " ".join(f"limit {k} {np.median([x[k][0] for x in v]):.3f} ms" for k in v[0]))
print("digests agree" if len(digs) == 1 else f"DIGESTS DIFFER: {digs}")
sys.exit(0 if len(digs) == 1 else 3)
