"""``/snapshotz`` ingestion: the cluster-autoscaler debugging snapshot as mirror input
(SURVEY.md §8f #4).

The reference's ``DebuggingSnapshotImpl`` (``CA/debuggingsnapshot/debugging_snapshot.go:
29-72``) is the JSON a running autoscaler serves on ``/snapshotz``: ``NodeList`` (each
``ClusterNode`` = a core/v1 Node and its Pods), ``UnscheduledPodsCanBeScheduled``,
``TemplateNodes`` (node group id -> ClusterNode), ``Error``, ``StartTimestamp``,
``EndTimestamp``.  ``load`` parses it into the host model (``k8s.py``: only the fields the
simulation reads — requests, ports, labels, taints, tolerations, node selectors and
required node affinity, owner references, annotations, deletion timestamps, volumes),
``dump`` writes the same shape back (``GetOutputBytes``, :115-130), and
``cluster_snapshot`` replays the ``NodeList`` into a ``ClusterSnapshot`` over the GPU
mirror, so a real cluster's state drives Estimate, FilterOutSchedulable, the sweep and
the utilization pass.  Host-side parsing only: no kernel is involved until the rows reach
the mirror.
"""
from __future__ import annotations

import datetime
import json
from dataclasses import dataclass, field
from typing import Optional

from .k8s import (Affinity, Container, ContainerPort, Node, NodeSelectorRequirement, NodeSelectorTerm,
                  OwnerReference, Pod, Quantity, Taint, Toleration)

_ZERO_TIME = "0001-01-01T00:00:00Z"          # Go's zero time.Time marshals to this


@dataclass
class ClusterNode:
    """debuggingsnapshot.ClusterNode (debugging_snapshot.go:29-32)."""
    Node: Optional[Node]
    Pods: list = field(default_factory=list)


@dataclass
class DebuggingSnapshot:
    """debuggingsnapshot.DebuggingSnapshotImpl (debugging_snapshot.go:64-72)."""
    NodeList: list = field(default_factory=list)
    UnscheduledPodsCanBeScheduled: list = field(default_factory=list)
    Error: str = ""
    StartTimestamp: str = _ZERO_TIME
    EndTimestamp: str = _ZERO_TIME
    TemplateNodes: dict = field(default_factory=dict)


# ---------------------------------------------------------------------------- time
def parse_time(s: Optional[str]) -> Optional[float]:
    """RFC 3339 (metav1.Time) -> seconds since the epoch."""
    if not s:
        return None
    s = s.replace("Z", "+00:00")
    if "." in s:                                   # Python wants at most 6 fractional digits
        head, rest = s.split(".", 1)
        k = 0
        while k < len(rest) and rest[k].isdigit():
            k += 1
        frac, tz = rest[:k], rest[k:]
        s = f"{head}.{frac[:6]}{tz}"
    return datetime.datetime.fromisoformat(s).timestamp()


def format_time(t: Optional[float]) -> Optional[str]:
    if t is None:
        return None
    return datetime.datetime.fromtimestamp(t, datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


# ---------------------------------------------------------------------------- objects
def _quantities(d: Optional[dict]) -> dict:
    return {k: Quantity(str(v)) for k, v in (d or {}).items()}


def _q_str(q: Quantity) -> str:
    v = q.v
    if v.denominator == 1:
        return str(v.numerator)
    m = v * 1000
    if m.denominator == 1:
        return f"{m.numerator}m"
    n = v * 10 ** 9
    return f"{n.numerator // n.denominator}n"


def _container(c: dict) -> Container:
    ports = [ContainerPort(host_port=int(p.get("hostPort", 0)), host_ip=p.get("hostIP", ""),
                           protocol=p.get("protocol", ""), container_port=int(p.get("containerPort", 0)))
             for p in c.get("ports") or []]
    return Container(requests=_quantities((c.get("resources") or {}).get("requests")), ports=ports)


def _requirement(r: dict) -> NodeSelectorRequirement:
    return NodeSelectorRequirement(r["key"], r["operator"], list(r.get("values") or []))


def _affinity(a: Optional[dict]) -> Optional[Affinity]:
    if not a:
        return None
    out = Affinity()
    na = a.get("nodeAffinity") or {}
    req = na.get("requiredDuringSchedulingIgnoredDuringExecution")
    if req is not None:
        out.required_terms = [NodeSelectorTerm([_requirement(e) for e in t.get("matchExpressions") or []],
                                               [_requirement(e) for e in t.get("matchFields") or []])
                              for t in req.get("nodeSelectorTerms") or []]
    out.pod_affinity = bool(a.get("podAffinity") or a.get("podAntiAffinity"))
    anti = a.get("podAntiAffinity") or {}
    out.required_anti_affinity = bool(anti.get("requiredDuringSchedulingIgnoredDuringExecution"))
    out.required_pod_affinity = bool((a.get("podAffinity") or {}).get("requiredDuringSchedulingIgnoredDuringExecution"))
    return out


def _volume_kind(v: dict) -> str:
    for k in v:
        if k != "name":
            return k
    return ""


def pod_from_json(d: dict) -> Pod:
    """core/v1 Pod JSON -> k8s.Pod."""
    md, spec, status = d.get("metadata") or {}, d.get("spec") or {}, d.get("status") or {}
    refs = [OwnerReference(r.get("kind", ""), r.get("name", ""), r.get("uid", ""), bool(r.get("controller", False)))
            for r in md.get("ownerReferences") or []]
    return Pod(
        name=md.get("name", ""), namespace=md.get("namespace", "") or "default", uid=md.get("uid", ""),
        labels=dict(md.get("labels") or {}), annotations=dict(md.get("annotations") or {}),
        containers=[_container(c) for c in spec.get("containers") or []],
        init_containers=[_container(c) for c in spec.get("initContainers") or []],
        overhead=_quantities(spec["overhead"]) if spec.get("overhead") is not None else None,
        node_name=spec.get("nodeName", ""),
        node_selector=dict(spec["nodeSelector"]) if spec.get("nodeSelector") is not None else None,
        affinity=_affinity(spec.get("affinity")),
        tolerations=[Toleration(t.get("key", ""), t.get("operator", ""), t.get("value", ""), t.get("effect", ""))
                     for t in spec.get("tolerations") or []],
        owner_refs=refs, volumes=[_volume_kind(v) for v in spec.get("volumes") or []],
        topology_spread=list(spec.get("topologySpreadConstraints") or []), phase=status.get("phase", "Running"),
        deletion_timestamp=parse_time(md.get("deletionTimestamp")), priority=spec.get("priority"),
        termination_grace_period_seconds=spec.get("terminationGracePeriodSeconds"),
        restart_policy=spec.get("restartPolicy", "Always") or "Always",
    )


def node_from_json(d: dict) -> Node:
    """core/v1 Node JSON -> k8s.Node (Status.Allocatable, Spec.Taints, Spec.Unschedulable)."""
    md, spec, status = d.get("metadata") or {}, d.get("spec") or {}, d.get("status") or {}
    return Node(name=md.get("name", ""), labels=dict(md.get("labels") or {}),
                taints=[Taint(t["key"], t.get("value", ""), t.get("effect", "")) for t in spec.get("taints") or []],
                allocatable=_quantities(status.get("allocatable")), unschedulable=bool(spec.get("unschedulable")))


def _container_json(c: Container) -> dict:
    out = {"name": "c", "resources": {"requests": {k: _q_str(v) for k, v in c.requests.items()}}}
    if c.ports:
        out["ports"] = [{k: v for k, v in (("containerPort", p.container_port), ("hostPort", p.host_port),
                                           ("hostIP", p.host_ip), ("protocol", p.protocol)) if v}
                        for p in c.ports]
    return out


def _req_json(r: NodeSelectorRequirement) -> dict:
    out = {"key": r.key, "operator": r.operator}
    if r.values:
        out["values"] = list(r.values)
    return out


def pod_to_json(p: Pod) -> dict:
    md = {"name": p.name, "namespace": p.namespace, "uid": p.uid}
    if p.labels:
        md["labels"] = dict(p.labels)
    if p.annotations:
        md["annotations"] = dict(p.annotations)
    if p.owner_refs:
        md["ownerReferences"] = [{"kind": r.kind, "name": r.name, "uid": r.uid, "controller": r.controller}
                                 for r in p.owner_refs]
    if p.deletion_timestamp is not None:
        md["deletionTimestamp"] = format_time(p.deletion_timestamp)
    spec = {"containers": [_container_json(c) for c in p.containers]}
    if p.init_containers:
        spec["initContainers"] = [_container_json(c) for c in p.init_containers]
    if p.overhead is not None:
        spec["overhead"] = {k: _q_str(v) for k, v in p.overhead.items()}
    if p.node_name:
        spec["nodeName"] = p.node_name
    if p.node_selector is not None:
        spec["nodeSelector"] = dict(p.node_selector)
    if p.affinity is not None and p.affinity.required_terms is not None:
        spec["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
            {"matchExpressions": [_req_json(e) for e in t.match_expressions],
             "matchFields": [_req_json(e) for e in t.match_fields]} for t in p.affinity.required_terms]}}}
    if p.tolerations:
        spec["tolerations"] = [{k: v for k, v in (("key", t.key), ("operator", t.operator), ("value", t.value),
                                                  ("effect", t.effect)) if v} for t in p.tolerations]
    if p.volumes:
        spec["volumes"] = [{"name": f"v{i}", k: {}} for i, k in enumerate(p.volumes)]
    if p.priority is not None:
        spec["priority"] = p.priority
    if p.termination_grace_period_seconds is not None:
        spec["terminationGracePeriodSeconds"] = p.termination_grace_period_seconds
    return {"metadata": md, "spec": spec, "status": {"phase": p.phase}}


def node_to_json(n: Node) -> dict:
    spec = {}
    if n.taints:
        spec["taints"] = [{"key": t.key, "value": t.value, "effect": t.effect} for t in n.taints]
    if n.unschedulable:
        spec["unschedulable"] = True
    md = {"name": n.name}
    if n.labels:
        md["labels"] = dict(n.labels)
    return {"metadata": md, "spec": spec,
            "status": {"allocatable": {k: _q_str(v) for k, v in n.allocatable.items()}}}


# ---------------------------------------------------------------------------- snapshot
def _cluster_node(d: dict) -> ClusterNode:
    node = d.get("Node")
    return ClusterNode(node_from_json(node) if node else None, [pod_from_json(p) for p in d.get("Pods") or []])


def load(data) -> DebuggingSnapshot:
    """Parse /snapshotz output (bytes, str or an already-decoded dict)."""
    d = json.loads(data) if isinstance(data, (bytes, str)) else data
    return DebuggingSnapshot(
        NodeList=[_cluster_node(c) for c in d.get("NodeList") or []],
        UnscheduledPodsCanBeScheduled=[pod_from_json(p) for p in d.get("UnscheduledPodsCanBeScheduled") or []],
        Error=d.get("Error", ""), StartTimestamp=d.get("StartTimestamp", _ZERO_TIME),
        EndTimestamp=d.get("EndTimestamp", _ZERO_TIME),
        TemplateNodes={k: _cluster_node(v) for k, v in (d.get("TemplateNodes") or {}).items()})


def dump(s: DebuggingSnapshot) -> bytes:
    """GetOutputBytes (debugging_snapshot.go:115-130): the snapshot as JSON."""
    def cn(c: ClusterNode) -> dict:
        return {"Node": node_to_json(c.Node) if c.Node else None, "Pods": [pod_to_json(p) for p in c.Pods]}
    out = {"NodeList": [cn(c) for c in s.NodeList],
           "UnscheduledPodsCanBeScheduled": [pod_to_json(p) for p in s.UnscheduledPodsCanBeScheduled]}
    if s.Error:
        out["Error"] = s.Error
    out.update({"StartTimestamp": s.StartTimestamp, "EndTimestamp": s.EndTimestamp,
                "TemplateNodes": {k: cn(v) for k, v in s.TemplateNodes.items()}})
    return json.dumps(out).encode()


def cluster_snapshot(s: DebuggingSnapshot, backend=None):
    """Replay NodeList into a ClusterSnapshot (node order = the snapshot's order; pods in
    their listed order), over the GPU mirror by default."""
    from .clustersnapshot import ClusterSnapshot
    snap = ClusterSnapshot(backend)
    for c in s.NodeList:
        if c.Node is not None:
            snap.AddNodeWithPods(c.Node, list(c.Pods))
    return snap
