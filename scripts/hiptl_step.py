"""Merged host-API / kernel timeline of one headline step from a rocprofv3 --hip-trace
--kernel-trace run: python scripts/hiptl_step.py <dir> [step_from_end]"""
import csv
import glob
import sys

d = sys.argv[1]
k_from_end = int(sys.argv[2]) if len(sys.argv) > 2 else 2
api = list(csv.DictReader(open(glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True)[0])))
ker = list(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])))
ev = []
for r in api:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api", r["Function"]))
for r in ker:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "gpu", r["Kernel_Name"].split("(")[0][:40]))
ev.sort()
inits = [e for e in ev if e[2] == "gpu" and "k_round_init" in e[3]]
t_init = inits[-k_from_end][0]
# the step's first API call: the hipSetDevice before that init
sets = [e for e in ev if e[2] == "api" and e[3] == "hipSetDevice" and e[0] < t_init]
t0 = sets[-1][0]
nxt = [e for e in ev if e[2] == "api" and e[3] == "hipSetDevice" and e[0] > t_init]
t1 = nxt[0][0] + 30000 if nxt else t_init + 1_000_000
for s, e, kind, name in ev:
    if t0 - 20000 <= s <= t1:
        print(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f} {'   ' if kind == 'api' else 'GPU'} {name}")
