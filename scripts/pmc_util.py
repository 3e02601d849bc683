"""Fixed-launch driver for rocprofv3 --pmc passes over the scale-down eligibility kernel:
3 launches of k_node_utilization on the C5-size table of bench.py's utilization leg."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from autoscaler_amd import native, workloads as W  # noqa: E402

nodes, off, pods, now = W.util_table(seed=11, n_nodes=15000, pods_per_node=20)
t = native.UtilTable(0, nodes, off, pods)
for _ in range(3):
    t.calculate(True, True, now, to_host=False)
t.close()
print("pmc_util ok", len(nodes), len(pods))
