"""Writes tests/golden/reference_cases.json: the known-answer tests of the reference.

The reference is Go (no toolchain in this container), so its tests
cannot be executed here.  Each case below transcribes one table row of a
reference test — its inputs (node/pod builders with the same arguments) and the
expected values the test asserts — with the file:line it comes from.  Quantities
are in the reference's units: cpu in millicores, memory in bytes, and the
estimator tests' makeNode/makePods memory in MiB (converted here).

Run:  python tests/golden/make_golden.py
"""
import json
import os

MIB = 1024 * 1024
EST = "CA/estimator/binpacking_estimator_test.go"
SCH = "CA/simulator/predicatechecker/schedulerbased_test.go"
CLU = "CA/simulator/cluster_test.go"
HNT = "CA/simulator/scheduling/hinting_simulator_test.go"


def est_node(cpu, mem_mib, name, zone):
    """makeNode (binpacking_estimator_test.go:83-103): pods 10, hostname + zone labels."""
    return {"name": name, "cpu": cpu, "mem": mem_mib * MIB, "pods": 10,
            "labels": {"kubernetes.io/hostname": name, "topology.kubernetes.io/zone": zone}}


def est_pods(cpu, mem_mib, hostport, count, max_skew=0, key=""):
    """makePods (binpacking_estimator_test.go:35-81): one pod object repeated."""
    p = {"name": "estimatee", "ns": "universe", "cpu": cpu, "mem": mem_mib * MIB, "labels": {"app": "estimatee"}}
    if hostport:
        p["hostport"] = hostport
    if max_skew > 0:       # :64-78: one DoNotSchedule constraint selecting app=estimatee
        p["topology_spread"] = [{"maxSkew": max_skew, "topologyKey": key, "whenUnsatisfiable": "DoNotSchedule",
                                 "labelSelector": {"matchLabels": {"app": "estimatee"}}}]
    return {"repeat": count, "pod": p}


def test_node(name, cpu, mem, **kw):
    """BuildTestNode (utils/test/test_utils.go:179-210): pods 100."""
    d = {"name": name, "cpu": cpu, "mem": mem, "pods": 100}
    d.update(kw)
    return d


def test_pod(name, cpu, mem, **kw):
    """BuildTestPod (utils/test/test_utils.go:36-68): UID = name, namespace default."""
    d = {"name": name, "cpu": cpu, "mem": mem}
    d.update(kw)
    return d


cases = []

# ---- estimator: TestBinpackingEstimate -------------------------------------
for name, line, cpu, mem, pods, max_nodes, en, ep in [
    ("simple resource-based binpacking", "118-125", 350 * 3 - 50, 2 * 1000, est_pods(350, 1000, 0, 10), 0, 5, 10),
    ("pods-per-node bound binpacking", "126-133", 10000, 20000, est_pods(10, 100, 0, 20), 0, 2, 20),
    ("hostport conflict forces pod-per-node", "134-141", 1000, 5000, est_pods(200, 1000, 5555, 8), 0, 8, 8),
    ("limiter cuts binpacking", "142-150", 1000, 5000, est_pods(500, 1000, 0, 20), 5, 5, 10),
]:
    cases.append({
        "id": f"estimate/{name}", "source": f"{EST}:{line},164-186", "kind": "estimate",
        "nodes": [est_node(100, 100, "oldnode", "zone-jupiter")],
        "template": est_node(cpu, mem, "template", "zone-mars"),
        "pods": pods, "max_nodes": max_nodes,
        "expect": {"node_count": en, "pod_count": ep},
    })
# the two topology-spread rows (:143-158) need PodTopologySpread: out of kernel scope.  The
# inputs are transcribed in full with the reference's expectation; the kernels must REJECT
# them (CA_EUNSUPPORTED -> UnsupportedByKernels, the Go path runs them), never count them.
for name, line, key, en, ep in [
        ("hostname topology spreading with maxSkew=2 forces 2 pods/node", "151-158", "kubernetes.io/hostname", 4, 8),
        ("zonal topology spreading with maxSkew=2 only allows 2 pods to schedule", "159-166",
         "topology.kubernetes.io/zone", 1, 2)]:
    cases.append({
        "id": f"estimate/{name}", "source": f"{EST}:{line},164-186", "kind": "estimate",
        "nodes": [est_node(100, 100, "oldnode", "zone-jupiter")],
        "template": est_node(1000, 5000, "template", "zone-mars"),
        "pods": est_pods(20, 100, 0, 8, 2, key), "max_nodes": 0,
        "expect": {"unsupported": True, "reference": {"node_count": en, "pod_count": ep},
                   "reason": "PodTopologySpread DoNotSchedule constraint (SURVEY §8a A12): routed to the Go path"},
    })

# ---- predicate checker: TestCheckPredicate ------------------------------------
n1000 = test_node("n1000", 1000, 2000000)
for name, line, sched, pod, err in [
    ("other pod - insuficient cpu", "47-53", [test_pod("p450", 450, 500000)], test_pod("p600", 600, 500000), True),
    ("other pod - ok", "54-60", [test_pod("p450", 450, 500000)], test_pod("p500", 500, 500000), False),
    ("empty - insuficient cpu", "61-67", [], test_pod("p8000", 8000, 0), True),
    ("empty - ok", "68-74", [], test_pod("p600", 600, 500000), False),
]:
    expect = {"error": err}
    if err:
        expect.update({"type": 0, "message": "Insufficient cpu",
                       "verbose_contains": "Insufficient cpu; predicateName=NodeResourcesFit"})
    cases.append({"id": f"check_predicates/{name}", "source": f"{SCH}:{line},73-91", "kind": "check_predicates",
                  "nodes": [dict(n1000, scheduled=sched)], "pod": pod, "node": "n1000", "expect": expect})

cases.append({
    "id": "check_predicates/debug info (taints)", "source": f"{SCH}:127-157", "kind": "check_predicates",
    "nodes": [test_node("n1", 1000, 2000000, taints=[["SomeTaint", "WhyNot?", "NoSchedule"],
                                                     ["RandomTaint", "JustBecause", "NoExecute"]])],
    "pod": test_pod("p1", 0, 0), "node": "n1",
    "expect": {"error": True, "message": "node(s) had untolerated taint {SomeTaint: WhyNot?}",
               "verbose_contains": "RandomTaint"},
})

# ---- predicate checker: TestFitsAnyNode ----------------------------------------
cases.append({
    "id": "fits_any_node/TestFitsAnyNode", "source": f"{SCH}:96-125", "kind": "fits_any_node",
    "nodes": [test_node("n1000", 1000, 2000000), test_node("n2000", 2000, 2000000)],
    "sequence": [
        {"pod": test_pod("p900", 900, 1000), "expect": ["n1000", "n2000"]},
        {"pod": test_pod("p1900", 1900, 1000), "expect": ["n2000"]},
        {"pod": test_pod("p2100", 2100, 1000), "expect": None},
    ],
})

# ---- removal simulator: TestFindNodesToRemove -----------------------------------
nodes = {"n1": test_node("n1", 1000, 2000000), "n2": test_node("n2", 1000, 2000000),
         "n3": test_node("n3", 1000, 2000000), "n4": test_node("n4", 1000, 2000000)}
pods = {
    "p1": test_pod("p1", 100, 100000, owner=["ReplicaSet", "rs"], node="n2"),
    "p2": test_pod("p2", 100, 100000, owner=["ReplicaSet", "rs"], node="n2"),
    "p3": test_pod("p3", 100, 100000, node="n3"),
    "p4": test_pod("p4", 1000, 100000, node="n4"),
}
for name, line, ps, cands, alln, to_remove, unremovable in [
    ("just an empty node, should be removed", "156-163", [], ["n1"], ["n1"], [["n1", []]], []),
    ("just a drainable node, but nowhere for pods to go to", "165-172", ["p1", "p2"], ["n2"], ["n2"], [],
     [["n2", "NoPlaceToMovePods", None, None]]),
    ("drainable node, and a mostly empty node that can take its pods", "174-181", ["p1", "p2", "p3"], ["n2", "n3"],
     ["n2", "n3"], [["n2", ["p1", "p2"]]], [["n3", "BlockedByPod", "p3", "NotReplicated"]]),
    ("drainable node, and a full node that cannot fit anymore pods", "183-190", ["p1", "p2", "p4"], ["n2"],
     ["n2", "n4"], [], [["n2", "NoPlaceToMovePods", None, None]]),
    ("4 nodes, 1 empty, 1 drainable", "192-199", ["p1", "p2", "p3", "p4"], ["n1", "n2"], ["n1", "n2", "n4", "n3"],
     [["n1", []], ["n2", ["p1", "p2"]]], []),
]:
    cases.append({
        "id": f"find_nodes_to_remove/{name}", "source": f"{CLU}:{line},198-216", "kind": "find_nodes_to_remove",
        "nodes": [nodes[n] for n in alln], "pods": [pods[p] for p in ps], "candidates": cands,
        "listers": {"ReplicaSet": [["default", "rs", 5]]},
        "delete_options": [True, True, 0],
        "expect": {"to_remove": to_remove, "unremovable": unremovable},
    })

cases.append({
    "id": "find_empty_nodes/TestFindEmptyNodes", "source": f"{CLU}:39-65", "kind": "find_empty_nodes",
    "nodes": [test_node(f"n{i}", 1000, 2000000) for i in range(4)],
    "pods": [test_pod("p1", 300, 500000, node="n1"),
             test_pod("p2", 300, 500000, node="n2", annotations={"kubernetes.io/config.mirror": ""})],
    "candidates": ["n0", "n1", "n2", "n3"],
    "expect": {"empty": ["n0", "n2", "n3"]},
})

# ---- hinting simulator: TestTrySchedulePods / TestPodSchedulesOnHintedNode -------
two = [test_node("n1", 1000, 2000000), test_node("n2", 1000, 2000000)]
p1 = test_pod("p1", 300, 500000, node="n1")
for name, line, new, acc, want in [
    ("two new pods, two nodes", "42-60", [test_pod("p2", 800, 500000), test_pod("p3", 500, 500000)], None,
     [["p2", "n2"], ["p3", "n1"]]),
    ("three new pods, two nodes, no fit", "61-80",
     [test_pod("p2", 800, 500000), test_pod("p3", 500, 500000), test_pod("p4", 700, 500000)], None,
     [["p2", "n2"], ["p3", "n1"]]),
    ("no new pods, two nodes", "81-92", [], None, []),
    ("two nodes, but only one acceptable", "93-111", [test_pod("p2", 500, 500000), test_pod("p3", 500, 500000)],
     ["n2"], [["p2", "n2"], ["p3", "n2"]]),
    ("two nodes, but only one acceptable, no fit", "112-129",
     [test_pod("p2", 500, 500000), test_pod("p3", 500, 500000)], ["n1"], [["p2", "n1"]]),
]:
    cases.append({
        "id": f"try_schedule_pods/{name}", "source": f"{HNT}:{line},132-157", "kind": "try_schedule_pods",
        "nodes": two, "pods": [p1], "new_pods": new, "acceptable": acc, "hints": {},
        "expect": {"statuses": want},
    })
for name, line, pn in [
    ("single hint", "170-174", {"p1": "n2"}),
    ("all on one node", "175-183", {"p1": "n2", "p2": "n2", "p3": "n2"}),
    ("spread across nodes", "184-192", {"p1": "n1", "p2": "n2", "p3": "n3"}),
    ("lots of pods", "193-207", {"p1": "n1", "p2": "n1", "p3": "n1", "p4": "n2", "p5": "n2", "p6": "n2",
                                 "p7": "n3", "p8": "n3", "p9": "n3"}),
]:
    cases.append({
        "id": f"hinted/{name}", "source": f"{HNT}:{line},205-232", "kind": "try_schedule_pods",
        "nodes": [test_node(n, 9999, 9999) for n in ("n1", "n2", "n3")], "pods": [],
        "new_pods": [test_pod(p, 1, 1) for p in pn], "acceptable": None, "hints": pn,
        "expect": {"statuses": [[p, n] for p, n in pn.items()]},
    })

# ---- FilterOutSchedulable: TestFilterOutSchedulable / BenchmarkFilterOutSchedulable ----
FOS = "CA/core/podlistprocessor/filter_out_schedulable_test.go"
fnode = [test_node("node", 2000, 100)]          # buildReadyTestNode("node", 2000, 100) (:33)
for name, line, existing, cand, want_sched, want_unsched in [
    ("single empty node, no pods", "43-46", [], [], [], []),
    ("single empty node, single schedulable pod", "47-56", [], [test_pod("pod", 500, 10)], ["pod"], []),
    ("single empty node, many schedulable pods", "57-70", [],
     [test_pod("pod1", 200, 10), test_pod("pod2", 500, 10), test_pod("pod3", 800, 10)], ["pod1", "pod2", "pod3"], []),
    ("single empty node, single unschedulable pod", "71-80", [], [test_pod("pod1", 3000, 10)], [], ["pod1"]),
    ("single empty node, various pods", "81-96", [],
     [test_pod("pod1", 200, 10), test_pod("pod2", 500, 10), test_pod("pod3", 1800, 10)], ["pod1", "pod2"], ["pod3"]),
    ("single empty node, some priority pods", "97-112", [],
     [test_pod("pod1", 200, 10), test_pod("pod2", 500, 10, priority=10), test_pod("pod3", 1800, 10, priority=20)],
     ["pod3", "pod1"], ["pod2"]),
    ("non-empty node with a single pods scheduled", "113-132", [test_pod("pod1", 500, 10, node="node")],
     [test_pod("pod2", 1000, 10), test_pod("pod3", 300, 10), test_pod("pod4", 300, 10)], ["pod2", "pod3"], ["pod4"]),
    ("non-empty node with many pods scheduled", "133-153",
     [test_pod("pod1", 500, 10, node="node"), test_pod("pod2", 1000, 10, node="node")],
     [test_pod("pod3", 1000, 10), test_pod("pod4", 300, 10), test_pod("pod5", 300, 10)], ["pod4"], ["pod3", "pod5"]),
]:
    cases.append({
        "id": f"filter_out_schedulable/{name}", "source": f"{FOS}:{line},146-191", "kind": "filter_out_schedulable",
        "nodes": fnode, "pods": existing, "candidates": cand,
        "expect": {"scheduled": want_sched, "unscheduled": want_unsched},
    })
# the benchmark's scenarios (:199-290): every pending pod (1000m, 2000000 B) fails on nodes of
# 2000m/200000 B holding 1000m/200000 B pods round-robin, so all stay pending
for name, nn, ns, npend in [("nothing", 1, 30, 1000), ("small", 10, 300, 1000), ("medium", 100, 3000, 1000),
                            ("large", 200, 200, 60000), ("1k", 1000, 1000, 12000)]:
    cases.append({
        "id": f"filter_out_schedulable/bench {name}", "source": f"{FOS}:199-290",
        "kind": "filter_out_schedulable_bench",
        "nodes": {"count": nn, "prefix": "n-", "cpu": 2000, "mem": 200000},
        "pods": {"count": ns, "prefix": "s-", "cpu": 1000, "mem": 200000},
        "candidates": {"count": npend, "prefix": "p-", "cpu": 1000, "mem": 2000000},
        "expect": {"still_pending": npend},
    })

# ---- scale-up: TestWillConsider*Pool* (orchestrator_test.go:304-404) ---------------------
# Options the expander receives (ComputeExpansionOption + Estimate per node group, limiter
# MaxNodesPerScaleUp = 0 in defaultOptions :57-63); node group templates are the groups'
# nodes (TemplateNodeInfoProvider over BuildTestNode + AddGpusToNode, no DaemonSet pods).
ORC = "CA/core/scaleup/orchestrator/orchestrator_test.go"


def orc_node(name, cpu, mem_mib, gpu, group):
    return {"name": name, "cpu": cpu, "mem": mem_mib * MIB, "pods": 100, "gpu": gpu, "group": group}


def orc_pod(name, cpu, mem_mib, gpu, node, tolerates):
    """buildTestPod (orchestrator_test.go:650-662): BuildTestPod + RequestGpuForPod + TolerateGpuForPod."""
    return {"name": name, "cpu": cpu, "mem": mem_mib * MIB, "gpu": gpu, "node": node, "tolerates_gpu": tolerates}


for name, line, nodes_, pods_, extra, options in [
    ("WillConsiderGpuAndStandardPoolForPodWhichDoesNotRequireGpu", "304-334",
     [orc_node("gpu-node-1", 2000, 1000, 1, "gpu-pool"), orc_node("std-node-1", 2000, 1000, 0, "std-pool")],
     [orc_pod("gpu-pod-1", 2000, 1000, 1, "gpu-node-1", True), orc_pod("std-pod-1", 2000, 1000, 0, "std-node-1", False)],
     [orc_pod("extra-std-pod", 2000, 1000, 0, "", True)], {"std-pool": 1, "gpu-pool": 1}),
    ("WillConsiderOnlyGpuPoolForPodWhichDoesRequiresGpu", "336-365",
     [orc_node("gpu-node-1", 2000, 1000, 1, "gpu-pool"), orc_node("std-node-1", 2000, 1000, 0, "std-pool")],
     [orc_pod("gpu-pod-1", 2000, 1000, 1, "gpu-node-1", True), orc_pod("std-pod-1", 2000, 1000, 0, "std-node-1", False)],
     [orc_pod("extra-gpu-pod", 2000, 1000, 1, "", True)], {"gpu-pool": 1}),
    ("WillConsiderAllPoolsWhichFitTwoPodsRequiringGpus", "367-404",
     [orc_node("gpu-1-node-1", 2000, 1000, 1, "gpu-1-pool"), orc_node("gpu-2-node-1", 2000, 1000, 2, "gpu-2-pool"),
      orc_node("gpu-4-node-1", 2000, 1000, 4, "gpu-4-pool"), orc_node("std-node-1", 2000, 1000, 0, "std-pool")],
     [orc_pod("gpu-pod-1", 2000, 1000, 1, "gpu-1-node-1", True), orc_pod("gpu-pod-2", 2000, 1000, 2, "gpu-2-node-1", True),
      orc_pod("gpu-pod-3", 2000, 1000, 4, "gpu-4-node-1", True), orc_pod("std-pod-1", 2000, 1000, 0, "std-node-1", False)],
     [orc_pod(f"extra-gpu-pod-{i}", 1, 1, 1, "", True) for i in (1, 2, 3)],
     {"gpu-1-pool": 3, "gpu-2-pool": 2, "gpu-4-pool": 1}),
]:
    cases.append({"id": f"expansion_options/{name}", "source": f"{ORC}:{line},478-576", "kind": "expansion_options",
                  "nodes": nodes_, "pods": pods_, "extra_pods": extra, "max_nodes": 0,
                  "expect": {"options": options}})

# ---- legacy scale-down: TestFindUnneededNodes (legacy_test.go:58-216) ------------------
# Five UpdateUnneededNodes calls over one ScaleDown; ng1 = {min 1, max 10, target 2};
# options: ScaleDownUtilizationThreshold 0.35, UnremovableNodeRecheckTimeout 5 min, every
# other option zero (NewScaleTestAutoscalingContext), NodeDeleteOptions zero; the rs lister
# holds ReplicaSet default/rs with 5 replicas (generateReplicaSets :1265-1279).
LEG = "CA/core/scaledown/legacy/legacy_test.go"
T0 = 1_700_000_000
leg_nodes = {
    "n1": test_node("n1", 1000, 10), "n2": test_node("n2", 1000, 10), "n3": test_node("n3", 1000, 10),
    "n4": test_node("n4", 10000, 10),
    "n5": test_node("n5", 1000, 10, annotations={"cluster-autoscaler.kubernetes.io/scale-down-disabled": "true"}),
    "n7": test_node("n7", 0, 10),
    "n8": test_node("n8", 1000, 10, taints=[["ToBeDeletedByClusterAutoscaler", str(T0 - 301), ""]]),
    "n9": test_node("n9", 1000, 10, taints=[["ToBeDeletedByClusterAutoscaler", str(T0 - 60), ""]]),
}
rs = ["ReplicaSet", "rs"]
leg_pods = {
    "p1": test_pod("p1", 100, 0, node="n1"), "p2": test_pod("p2", 300, 0, node="n2", owner=rs),
    "p3": test_pod("p3", 400, 0, node="n3", owner=rs), "p4": test_pod("p4", 2000, 0, node="n4", owner=rs),
    "p5": test_pod("p5", 100, 0, node="n5", owner=rs), "p6": test_pod("p6", 500, 0, node="n7", owner=rs),
}
all8 = ["n1", "n2", "n3", "n4", "n5", "n7", "n8", "n9"]
cases.append({
    "id": "update_unneeded_nodes/TestFindUnneededNodes", "source": f"{LEG}:58-216", "kind": "update_unneeded_nodes",
    "nodes": leg_nodes, "pods": leg_pods, "groups": {"ng1": [1, 10, 2, all8]}, "now": T0,
    "options": {"threshold": 0.35, "recheck_timeout": 300.0, "non_empty_candidates": 0, "pool_ratio": 0.0,
                "pool_min": 0},
    "listers": {"ReplicaSet": [["default", "rs", 5]]},
    "steps": [
        {"line": "150-166", "nodes": all8, "pods": ["p1", "p2", "p3", "p4", "p5", "p6"], "candidates": all8,
         "expect": {"unneeded": ["n2", "n7", "n8"], "util_found": ["n1", "n2", "n3", "n4", "n7", "n8"],
                    "util_missing": ["n5", "n6", "n9"]}},
        {"line": "168-184", "reset_unremovable": True, "preset_unneeded": ["n1", "n2", "n3", "n4"],
         "nodes": ["n1", "n2", "n3", "n4"], "pods": ["p1", "p2", "p3", "p4"], "candidates": ["n1", "n2", "n3", "n4"],
         "expect": {"unneeded": ["n2"], "util_found": ["n1", "n2", "n3", "n4"], "util_missing": ["n5", "n6"]}},
        {"line": "186-192", "reset_unremovable": True, "nodes": ["n1", "n2", "n3", "n4"],
         "pods": ["p1", "p2", "p3", "p4"], "candidates": ["n1", "n3", "n4"], "expect": {"unneeded": []}},
        {"line": "194-202", "nodes": ["n1"], "pods": [], "candidates": ["n1"],
         "expect": {"unneeded": [], "unremovable_count": 1}},
        {"line": "204-215", "nodes": ["n1"], "pods": [], "candidates": ["n1"], "time_offset": 301.0,
         "expect": {"unneeded": ["n1"], "unremovable_count": 0}},
    ],
})

# ---- planner: TestUpdateClusterState / TestUpdateClusterStatUnneededNodesLimit -------
# Planner.UpdateClusterState with canPersist=true (planner.go:103-126,252-296): nodes are
# BuildTestNode(name, cpu, 10); nodeUndergoingDeletion adds the ToBeDeleted NoSchedule taint
# (planner_test.go:661-666); the ReplicaSet lister holds generateReplicaSets("rs", 5) unless
# a case says otherwise (:474-476, :619-657: spec replicas, status replicas).  Destinations
# and candidates are all nodes (:506); the eligibility checker is the fake one (:688-705).
PLN = "CA/core/scaledown/planner/planner_test.go"
TBD = ["ToBeDeletedByClusterAutoscaler", "", "NoSchedule"]


def pl_node(name, cpu, deleting=False):
    return test_node(name, cpu, 10, **({"taints": [TBD]} if deleting else {}))


def pl_pod(name, cpu, node, kind="rs", owner="rs"):
    d = test_pod(name, cpu, 1, node=node)
    if kind == "rs":
        d["owner"] = ["ReplicaSet", owner]
    elif kind == "ds":
        d["owner"] = ["DaemonSet", "ds"]
    elif kind == "static":
        d["annotations"] = {"kubernetes.io/config.source": "file"}
    elif kind == "mirror":
        d["annotations"] = {"kubernetes.io/config.mirror": "mirror"}
    return d


RS5 = {"rs": [5, 0]}
for name, line, nodes, pods, evictions, eligible, unneeded, unremovable, rsets in [
    ("empty nodes, all eligible", "58-67", [pl_node("n1", 1000), pl_node("n2", 1000), pl_node("n3", 1000)], [], [],
     ["n1", "n2", "n3"], ["n1", "n2", "n3"], [], RS5),
    ("empty nodes, some eligible", "68-79", [pl_node("n1", 1000), pl_node("n2", 1000), pl_node("n3", 1000)], [], [],
     ["n1", "n2"], ["n1", "n2"], ["n3"], RS5),
    ("empty nodes, none eligible", "80-91", [pl_node("n1", 1000), pl_node("n2", 1000), pl_node("n3", 1000)], [], [],
     [], [], ["n1", "n2", "n3"], RS5),
    ("single utilised node, not eligible", "92-104", [pl_node("n1", 1000)], [pl_pod("p1", 500, "n1")], [],
     ["n1"], [], ["n1"], RS5),
    ("pods cannot schedule on node undergoing deletion, not eligible", "105-119",
     [pl_node("n1", 1000), pl_node("n2", 1000, True)], [pl_pod("p1", 500, "n1"), pl_pod("p2", 500, "n1")], [],
     ["n1"], [], ["n1", "n2"], RS5),
    ("pods can schedule on non-eligible node, eligible", "120-134", [pl_node("n1", 1000), pl_node("n2", 1000)],
     [pl_pod("p1", 500, "n1"), pl_pod("p2", 500, "n1")], [], ["n1"], ["n1"], ["n2"], RS5),
    ("pods can schedule on eligible node, eligible", "135-149", [pl_node("n1", 1000), pl_node("n2", 1000)],
     [pl_pod("p1", 500, "n1"), pl_pod("p2", 500, "n1")], [], ["n1", "n2"], ["n1"], ["n2"], RS5),
    ("pods cannot schedule anywhere, not eligible", "150-166",
     [pl_node("n1", 2000), pl_node("n2", 1000), pl_node("n3", 500)],
     [pl_pod("p1", 1000, "n1"), pl_pod("p2", 1000, "n1"), pl_pod("p3", 1000, "n2")], [],
     ["n1", "n2"], [], ["n1", "n2", "n3"], RS5),
    ("all pods from multiple nodes can schedule elsewhere, all eligible", "167-184",
     [pl_node("n1", 1000), pl_node("n2", 1000), pl_node("n3", 2000)],
     [pl_pod("p1", 500, "n1"), pl_pod("p2", 500, "n1"), pl_pod("p3", 500, "n2"), pl_pod("p4", 500, "n2")], [],
     ["n1", "n2"], ["n1", "n2"], ["n3"], RS5),
    ("some pods from multiple nodes can schedule elsewhere, some eligible", "185-202",
     [pl_node("n1", 2000), pl_node("n2", 1000), pl_node("n3", 1000)],
     [pl_pod("p1", 1000, "n1"), pl_pod("p2", 1000, "n1"), pl_pod("p3", 500, "n2"), pl_pod("p4", 500, "n2")], [],
     ["n1", "n2"], ["n2"], ["n1", "n3"], RS5),
    ("no pods from multiple nodes can schedule elsewhere, no eligible", "203-220",
     [pl_node("n1", 1000), pl_node("n2", 1000), pl_node("n3", 500)],
     [pl_pod("p1", 500, "n1"), pl_pod("p2", 500, "n1"), pl_pod("p3", 500, "n2"), pl_pod("p4", 500, "n2")], [],
     ["n1", "n2"], [], ["n1", "n2", "n3"], RS5),
    ("recently evicted RS pod, not eligible", "221-235", [pl_node("n1", 1000), pl_node("n2", 2000, True)], [],
     [pl_pod("p1", 500, "n2")], ["n1"], [], ["n1", "n2"], RS5),
    ("recently evicted pod without owner, not eligible", "236-249", [pl_node("n1", 1000)], [],
     [pl_pod("p1", 1000, "", kind="none")], ["n1"], [], ["n1"], RS5),
    ("recently evicted static pod, eligible", "250-264", [pl_node("n1", 1000), pl_node("n2", 2000, True)], [],
     [pl_pod("p1", 500, "n2", kind="static")], ["n1"], ["n1"], ["n2"], RS5),
    ("recently evicted mirror pod, eligible", "265-279", [pl_node("n1", 1000), pl_node("n2", 2000, True)], [],
     [pl_pod("p1", 500, "n2", kind="mirror")], ["n1"], ["n1"], ["n2"], RS5),
    ("recently evicted DS pod, eligible", "280-294", [pl_node("n1", 1000), pl_node("n2", 2000, True)], [],
     [pl_pod("p1", 500, "n2", kind="ds")], ["n1"], ["n1"], ["n2"], RS5),
    ("recently evicted pod can schedule on non-eligible node, eligible", "295-310",
     [pl_node("n1", 1000), pl_node("n2", 1000), pl_node("n3", 1000, True)], [], [pl_pod("p1", 500, "n3")],
     ["n1"], ["n1"], ["n2", "n3"], RS5),
    ("recently evicted pod can schedule on eligible node, eligible", "311-326",
     [pl_node("n1", 1000), pl_node("n2", 1000), pl_node("n3", 1000, True)], [], [pl_pod("p1", 500, "n3")],
     ["n1", "n2"], ["n1"], ["n2", "n3"], RS5),
    ("recently evicted pod too large to schedule anywhere, all eligible", "327-342",
     [pl_node("n1", 1000), pl_node("n2", 1000), pl_node("n3", 2000, True)], [], [pl_pod("p1", 2000, "n3")],
     ["n1", "n2"], ["n1", "n2"], ["n3"], RS5),
    ("all recently evicted pod got rescheduled, all eligible", "343-360",
     [pl_node("n1", 1000), pl_node("n2", 1000), pl_node("n3", 2000, True)], [],
     [pl_pod("p1", 1000, "n3", owner="rs1"), pl_pod("p2", 1000, "n3", owner="rs1")],
     ["n1", "n2"], ["n1", "n2"], ["n3"], {"rs1": [2, 2], "rs": [5, 0]}),
    ("some recently evicted pod got rescheduled, some eligible", "361-378",
     [pl_node("n1", 1000), pl_node("n2", 1000), pl_node("n3", 2000, True)], [],
     [pl_pod("p1", 1000, "n3", owner="rs1"), pl_pod("p2", 1000, "n3", owner="rs1")],
     ["n1", "n2"], ["n1"], ["n2", "n3"], {"rs1": [2, 1], "rs": [5, 0]}),
    ("no recently evicted pod got rescheduled, no eligible", "379-396",
     [pl_node("n1", 1000), pl_node("n2", 1000), pl_node("n3", 2000, True)], [],
     [pl_pod("p1", 1000, "n3", owner="rs1"), pl_pod("p2", 1000, "n3", owner="rs1")],
     ["n1", "n2"], [], ["n1", "n2", "n3"], {"rs1": [2, 0], "rs": [5, 0]}),
    ("all scheduled and recently evicted pods can schedule elsewhere, all eligible", "397-417",
     [pl_node("n1", 1000), pl_node("n2", 1000), pl_node("n3", 1000), pl_node("n4", 2000, True)],
     [pl_pod("p1", 250, "n1")], [pl_pod("p2", 250, "n4"), pl_pod("p3", 250, "n4")],
     ["n1", "n2"], ["n1", "n2"], ["n3", "n4"], RS5),
    ("some scheduled and recently evicted pods can schedule elsewhere, some eligible", "418-438",
     [pl_node("n1", 1000), pl_node("n2", 1000), pl_node("n3", 1000), pl_node("n4", 2000, True)],
     [pl_pod("p1", 500, "n1")], [pl_pod("p2", 500, "n4"), pl_pod("p3", 500, "n4")],
     ["n1", "n2"], ["n1"], ["n2", "n3", "n4"], RS5),
    ("scheduled and recently evicted pods take all capacity, no eligible", "439-459",
     [pl_node("n1", 1000), pl_node("n2", 1000), pl_node("n3", 1000), pl_node("n4", 2000, True)],
     [pl_pod("p1", 1000, "n1")], [pl_pod("p2", 1000, "n4"), pl_pod("p3", 1000, "n4")],
     ["n1", "n2"], [], ["n1", "n2", "n3", "n4"], RS5),
]:
    cases.append({"id": f"planner/{name}", "source": f"{PLN}:{line},471-512", "kind": "planner",
                  "nodes": nodes, "pods": pods, "evictions": evictions, "eligible": eligible,
                  "replicas": rsets, "listers": {"ReplicaSet": [["default", k, v[0]] for k, v in rsets.items()]},
                  "expect": {"unneeded": unneeded, "unremovable": unremovable}})

for name, line, prev, maxp, unneeded_s, interval_s, want in [
    ("no unneeded, default settings", "526-534", 0, 10, 60, 10, 20),
    ("some unneeded, default settings", "535-543", 3, 10, 60, 10, 23),
    ("max unneeded, default settings", "544-552", 70, 10, 60, 10, 70),
    ("too many unneeded, default settings", "553-561", 77, 10, 60, 10, 70),
    ("instant kill nodes", "562-570", 0, 10, 0, 10, 20),
    ("quick loops", "571-579", 13, 10, 60, 1, 33),
    ("slow loops", "580-588", 13, 10, 60, 30, 30),
]:
    cases.append({"id": f"planner_limit/{name}", "source": f"{PLN}:{line},590-614", "kind": "planner_limit",
                  "n_nodes": 100, "previously_unneeded": prev, "max_parallelism": maxp,
                  "unneeded_time_s": unneeded_s, "update_interval_s": interval_s, "expect": {"unneeded_count": want}})

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_cases.json")
    with open(out, "w") as f:
        json.dump({"generated_by": "tests/golden/make_golden.py", "cases": cases}, f, indent=1)
    print(f"wrote {len(cases)} cases to {out}")
