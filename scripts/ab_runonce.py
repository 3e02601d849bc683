"""A/B of two builds of the library on the C5 RunOnce loop's legs: alternating processes,
each running 5 loops (fork, runonce.run, revert) and printing the median of the last 4 per
leg.  Usage: python scripts/ab_runonce.py LIB_A LIB_B [LIB ...] [rounds]"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import json, sys
sys.path.insert(0, %r)
import numpy as np
from autoscaler_amd import native, runonce, workloads as W
w = runonce.c5_runonce()
m = native.Mirror(0)
W.load_filter(m, w.filt)
util = runonce.DeviceUtil(0)
expand = runonce.DeviceExpansion()
runs = []
for _ in range(5):
    m.fork()
    runs.append(runonce.run(m, util, w, expand_fn=expand))
    m.revert()
print(json.dumps({k: float(np.median([r.ms[k] for r in runs[1:]])) for k in runs[-1].ms}))
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
        d = json.loads(out.stdout.strip().splitlines()[-1])
        res[lib].append(d)
        print(f"round {r} {lib}: " + " ".join(f"{k} {v:.3f}" for k, v in d.items()), flush=True)
for lib, v in res.items():
    print(f"{lib}: median " + " ".join(f"{k} {np.median([x[k] for x in v]):.3f}" for k in v[0]))
