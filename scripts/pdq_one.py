"""One device Go sort of the heaviest C2 group's ranks per store (for rocprofv3 counter
passes: scripts/gpu_job.sh pmc "<counters>|scripts/pdq_one.py [store ...]")."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autoscaler_amd import native, workloads as W  # noqa: E402

w = W.c2()
p = w.table.pods
g = int(np.argmax(np.diff(w.group_off)))
idx = w.pod_idx[w.group_off[g]:w.group_off[g + 1]]
ac = float(w.templates[g]["node"]["alloc_milli_cpu"]); am = float(w.templates[g]["node"]["alloc_memory"])
score = p["score_milli_cpu"][idx] / ac + p["score_memory"][idx] / am
ranks = np.unique(-score, return_inverse=True)[1].astype(np.uint32)
for st in [int(a) for a in sys.argv[1:]] or [1]:
    native.go_sort_ranks(ranks, store=st)
print("ok", len(ranks))
