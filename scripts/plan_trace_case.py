import os, sys
sys.path.insert(0, "tests"); sys.path.insert(0, "oracle"); sys.path.insert(0, ".")
os.environ.setdefault("CASIM_PLAN_TRACE", "5")
os.environ.setdefault("CASIM_TEST_HOOKS", "1")
import numpy as np
from plangen import rand_plan_case
from autoscaler_amd import native
import pyoracle
case = rand_plan_case(7, n_nodes=10, pods_per_node=4, n_pdbs=2)
print("cands", case.cands, "off", case.off, "moves", case.moves, "hints", case.hints[case.moves], "L0", case.L0)
print("mask", case.mask)
p = case.table.pods
print("pods cpu", p["req_milli_cpu"][case.moves], "mem", p["req_memory"][case.moves], "eph", p["req_ephemeral"][case.moves], "flags", [hex(x) for x in p["flags"][case.moves]])
print("nodes", case.node_recs[["alloc_milli_cpu","alloc_memory","alloc_ephemeral","alloc_pods","flags"]])
o = pyoracle.OracleState(); case.load(o); po = case.plan(o)
print("oracle", po.results, po.moves)
m = native.Mirror(0); case.load(m); pm = case.plan(m)
print("gpu", pm.results, pm.moves)
