"""Writes tests/golden/intern_fixtures.json: API objects (core/v1 JSON, as a Go shim
unmarshals them) -> the include/casim.h records the interning must produce.

The shim that binds libcasim from cluster-autoscaler has to restate the interning
(autoscaler_amd/intern.py: taint classes, label pairs/keys, Gt/Lt keys, host-port triples
with the 0.0.0.0 wildcard, scalar resources, node names, selector programs, PreFilter
NodeNames, TPU requests, scope flags).  These fixtures are the shared check: each case
lists the objects in observation order, the universes that result (ids = list index), and
every encoded ca_node_spec / ca_pod_spec / ca_template field, selector term and requirement.

Run:  python tests/golden/make_intern_fixtures.py
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from autoscaler_amd import snapshotz  # noqa: E402
from autoscaler_amd.intern import Interner  # noqa: E402

GI = 1024 ** 3


def node(name, cpu="4", mem="16Gi", labels=None, taints=None, unschedulable=False, extra=None):
    alloc = {"cpu": cpu, "memory": mem, "pods": "110", "ephemeral-storage": "100Gi"}
    alloc.update(extra or {})
    spec = {"taints": taints} if taints else {}
    if unschedulable:
        spec["unschedulable"] = True
    return {"metadata": {"name": name, "labels": labels or {}}, "spec": spec, "status": {"allocatable": alloc}}


def pod(name, requests=None, **spec_extra):
    req = {"cpu": "250m", "memory": "512Mi"} if requests is None else requests
    containers = [{"name": "c", "resources": {"requests": req}}]
    spec = {"containers": containers}
    meta = {"name": name, "namespace": "default", "uid": name}
    meta.update(spec_extra.pop("metadata", {}))
    spec.update(spec_extra)
    return {"metadata": meta, "spec": spec}


CASES = [
    {"name": "resources, init containers, overhead, extended and TPU resources",
     "nodes": [node("n1", extra={"nvidia.com/gpu": "4", "cloud-tpus.google.com/v3": "8", "hugepages-2Mi": "1Gi"})],
     "pods": [
         pod("plain"),
         pod("init", initContainers=[{"name": "i", "resources": {"requests": {"cpu": "2", "memory": "100Mi"}}}]),
         pod("overhead", overhead={"cpu": "100m", "memory": "64Mi"}),
         pod("gpu", requests={"cpu": "1", "memory": "1Gi", "nvidia.com/gpu": "2"}),
         pod("tpu", requests={"cpu": "1", "cloud-tpus.google.com/v3": "8"}),
         pod("zero", requests={}),
         pod("milli-round", requests={"cpu": "0.0005", "memory": "1.5"}),
     ]},
    {"name": "taints and tolerations",
     "nodes": [node("t1", taints=[{"key": "dedicated", "value": "ml", "effect": "NoSchedule"},
                                  {"key": "spot", "value": "", "effect": "NoExecute"},
                                  {"key": "soft", "value": "x", "effect": "PreferNoSchedule"}]),
               node("t2", taints=[{"key": "dedicated", "value": "web", "effect": "NoSchedule"}], unschedulable=True)],
     "pods": [
         pod("none"),
         pod("exists", tolerations=[{"key": "dedicated", "operator": "Exists"}]),
         pod("equal", tolerations=[{"key": "dedicated", "operator": "Equal", "value": "ml", "effect": "NoSchedule"}]),
         pod("all", tolerations=[{"operator": "Exists"}]),
         pod("unsched", tolerations=[{"key": "node.kubernetes.io/unschedulable", "operator": "Exists",
                                      "effect": "NoSchedule"}]),
     ]},
    {"name": "node selectors and required node affinity",
     "nodes": [node("a1", labels={"zone": "a", "gen": "5", "ssd": "true"}),
               node("a2", labels={"zone": "b", "gen": "x"})],
     "pods": [
         pod("selector", nodeSelector={"zone": "a", "ssd": "true"}),
         pod("in-notin", affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
             "nodeSelectorTerms": [{"matchExpressions": [{"key": "zone", "operator": "In", "values": ["a", "c"]},
                                                         {"key": "ssd", "operator": "NotIn", "values": ["false"]}]},
                                   {"matchExpressions": [{"key": "gen", "operator": "Gt", "values": ["4"]}]}]}}}),
         pod("exists", affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
             "nodeSelectorTerms": [{"matchExpressions": [{"key": "ssd", "operator": "Exists"},
                                                         {"key": "gpu", "operator": "DoesNotExist"}]}]}}}),
         pod("fields", affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
             "nodeSelectorTerms": [{"matchFields": [{"key": "metadata.name", "operator": "In", "values": ["a2"]}]}]}}}),
         pod("bad-term", affinity={"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
             "nodeSelectorTerms": [{"matchExpressions": [{"key": "gen", "operator": "Lt", "values": ["x"]}]},
                                   {"matchExpressions": []}]}}}),
         pod("hostname", nodeSelector={"kubernetes.io/hostname": "a1"}),
         pod("node-name", nodeName="a2"),
     ]},
    {"name": "host ports",
     "nodes": [node("p1")],
     "pods": [
         pod("tcp80", containers=[{"name": "c", "ports": [{"containerPort": 80, "hostPort": 8080}],
                                   "resources": {"requests": {"cpu": "100m"}}}]),
         pod("ip80", containers=[{"name": "c", "ports": [{"containerPort": 80, "hostPort": 8080,
                                                          "hostIP": "10.0.0.1"}],
                                  "resources": {"requests": {"cpu": "100m"}}}]),
         pod("udp80", containers=[{"name": "c", "ports": [{"containerPort": 80, "hostPort": 8080,
                                                           "protocol": "UDP"}],
                                   "resources": {"requests": {"cpu": "100m"}}}]),
     ]},
    {"name": "kernel scope and controllers",
     "nodes": [node("s1")],
     "pods": [
         pod("spread", topologySpreadConstraints=[{"maxSkew": 1, "topologyKey": "zone",
                                                   "whenUnsatisfiable": "DoNotSchedule",
                                                   "labelSelector": {"matchLabels": {"app": "x"}}}]),
         pod("spread-soft", topologySpreadConstraints=[{"maxSkew": 1, "topologyKey": "zone",
                                                        "whenUnsatisfiable": "ScheduleAnyway"}]),
         pod("anti", affinity={"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
             {"labelSelector": {"matchLabels": {"app": "x"}}, "topologyKey": "kubernetes.io/hostname"}]}}),
         pod("pvc", volumes=[{"name": "d", "persistentVolumeClaim": {"claimName": "c"}}]),
         pod("emptydir", volumes=[{"name": "d", "emptyDir": {}}]),
         pod("ds", metadata={"ownerReferences": [{"kind": "DaemonSet", "name": "d", "uid": "ds-uid",
                                                  "controller": True}]}),
         pod("ds-annot", metadata={"annotations": {"cluster-autoscaler.kubernetes.io/daemonset-pod": "true"}}),
         pod("rs-a", metadata={"labels": {"app": "a"}, "ownerReferences": [{"kind": "ReplicaSet", "name": "r",
                                                                            "uid": "rs-uid", "controller": True}]}),
         pod("rs-b", metadata={"labels": {"app": "a"}, "ownerReferences": [{"kind": "ReplicaSet", "name": "r",
                                                                            "uid": "rs-uid", "controller": True}]}),
     ],
     "templates": [{"node": node("tmpl"), "pods": [pod("tds", metadata={"ownerReferences": [
         {"kind": "DaemonSet", "name": "d", "uid": "d2", "controller": True}]})]}]},
]


def rec_dict(rec) -> dict:
    out = {}
    for name in rec.dtype.names:
        v = rec[name]
        out[name] = rec_dict(v) if v.dtype.names else (v.tolist() if isinstance(v, np.ndarray) else v.item())
    return out


def build(case: dict) -> dict:
    nodes = [snapshotz.node_from_json(n) for n in case["nodes"]]
    pods = [snapshotz.pod_from_json(p) for p in case["pods"]]
    tmpls = [(snapshotz.node_from_json(t["node"]), [snapshotz.pod_from_json(p) for p in t["pods"]])
             for t in case.get("templates", [])]
    it = Interner(nodes, pods, tmpls)
    recs = it.encode_nodes(nodes)
    table = it.encode_pods(pods)
    return {
        "universes": {
            "taints": [list(k) for k in it.taints.ids], "label_pairs": [list(k) for k in it.pairs.ids],
            "label_keys": list(it.keys.ids), "int_keys": list(it.int_keys.ids), "ports": [list(k) for k in it.ports.ids],
            "scalars": list(it.scalars.ids), "names": list(it.names),
        },
        "nodes": [rec_dict(r) for r in recs],
        "pods": [rec_dict(r) for r in table.pods],
        "terms": [rec_dict(r) for r in table.terms],
        "reqs": [rec_dict(r) for r in table.reqs],
        "prefilter_names": table.names.tolist(),
        "templates": [rec_dict(it.encode_template(n, ps)) for n, ps in tmpls],
    }


def main():
    out = {"generated_by": "tests/golden/make_intern_fixtures.py", "cases": []}
    for c in CASES:
        out["cases"].append({"name": c["name"], "input": {k: c[k] for k in ("nodes", "pods", "templates") if k in c},
                             "expect": build(c)})
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "intern_fixtures.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {len(out['cases'])} cases")


if __name__ == "__main__":
    main()
