"""Summarise one rocprofv3 --pmc pass of SQ counters (python scripts/pmc_sq.py <dir>):
per kernel, per launch: wave cycles split into parked (SQ_WAIT_ANY: s_waitcnt / barrier),
issue-stalled (SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY), and the instruction mix
(MI355X_MICROARCH.md, rocprofv3 PMC slots: the three cycle buckets are disjoint and count
quad-cycles)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1]
per = defaultdict(lambda: defaultdict(float))
launches = defaultdict(set)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        name = name[5:] if name.startswith("void ") else name
        name = name.split("<")[0]
        disp = r.get("Dispatch_Id", r.get("Correlation_Id", ""))
        per[name][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[name].add(disp)
out = {}
for name, c in per.items():
    n = max(len(launches[name]), 1)
    wc = c.get("SQ_WAVE_CYCLES", 0.0)
    rec = {k: v / n for k, v in c.items()}
    rec["launches"] = n
    if wc > 0:
        rec["share_parked"] = c.get("SQ_WAIT_ANY", 0.0) / wc
        rec["share_issue_stalled"] = c.get("SQ_WAIT_INST_ANY", 0.0) / wc
        rec["share_issuing"] = c.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
    out[name] = rec
json.dump({"source": "rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY "
                     "SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS over scripts/pmc_step.py "
                     "PMC_LEGS=all; values per launch", "kernels": out}, sys.stdout, indent=1)
