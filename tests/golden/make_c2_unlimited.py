"""Writes tests/golden/c2_unlimited.json: the CPU restatement's Estimate of the full C2
batch with an UNLIMITED limiter (maxNodes = 0, threshold_based_limiter.go:49-52; BASELINE
C2 row, the second limiter setting).  The oracle takes ~2 min on one core (9.1e9 filter
evaluations), too long for a GPU test, so its results are committed: every group's
ca_estimate_result fields, the batch lastIndex, and a CRC-32 of each group's scheduled
pod list (processing order).  tests/test_gpu_parity.py compares the device against it.

Run:  python tests/golden/make_c2_unlimited.py
"""
import json
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from autoscaler_amd import workloads as W  # noqa: E402
import pyoracle  # noqa: E402

FIELDS = ["node_count", "n_scheduled", "nodes_added", "last_index_in", "last_index_out", "status", "evals"]


def summarize(results, sched_pod, group_off, last_index):
    out = {"last_index": int(last_index), "groups": []}
    for g in range(len(results)):
        r = results[g]
        a, n = int(group_off[g]), int(r["n_scheduled"])
        out["groups"].append({**{f: int(r[f]) for f in FIELDS},
                              "sched_crc32": zlib.crc32(np.ascontiguousarray(sched_pod[a:a + n], np.int32).tobytes())})
    return out


if __name__ == "__main__":
    w = W.c2()
    o = pyoracle.OracleState()
    W.load_estimate(o, w)
    r = o.estimate(w.table, w.group_off, w.pod_idx, w.templates, 0, 0)
    doc = {"generated_by": "tests/golden/make_c2_unlimited.py", "workload": "C2 (workloads.c2 defaults), max_nodes=0",
           **summarize(r.results, r.sched_pod, w.group_off, r.last_index)}
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "c2_unlimited.json"), "w") as f:
        json.dump(doc, f, indent=0)
    print("groups", len(doc["groups"]), "evals", sum(g["evals"] for g in doc["groups"]))
