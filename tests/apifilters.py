"""Independent API-level restatement of the six in-kernel filters, evaluated on the
k8s objects directly (strings, maps) — no interning.  Used to cross-check the
interner + the oracle's bitset evaluation on random clusters.

Follows SF/plugins/{nodeunschedulable,nodename,tainttoleration,nodeaffinity,
nodeports,noderesources}, component-helpers nodeaffinity.go and labels/selector.go.
"""
from __future__ import annotations

import math
from fractions import Fraction

from autoscaler_amd.intern import is_qualified_name, is_valid_label_value, is_scalar_resource, parse_int64
from autoscaler_amd.k8s import Quantity, Taint


def _q(v):
    return v if isinstance(v, Quantity) else Quantity(v)


def request(pod):
    """max(sum containers, each init) + overhead, per resource name."""
    def add(d, rl, mx=False):
        for k, v in rl.items():
            if k == "pods":
                continue
            q = _q(v)
            val = q.milli_value() if k == "cpu" else q.value()
            if k not in ("cpu", "memory", "ephemeral-storage") and not is_scalar_resource(k):
                continue
            d[k] = max(d.get(k, 0), val) if mx else d.get(k, 0) + val
    r = {}
    for c in pod.containers:
        add(r, c.requests)
    for c in pod.init_containers:
        add(r, c.requests, mx=True)
    if pod.overhead is not None:
        add(r, pod.overhead)
    return r


def tolerates(t, taint) -> bool:
    if t.effect and t.effect != taint.effect:
        return False
    if t.key and t.key != taint.key:
        return False
    if t.operator in ("", "Equal"):
        return t.value == taint.value
    return t.operator == "Exists"


def req_match(r, labels) -> bool | None:
    """labels.Requirement.Matches; None marks a parse error (term never matches)."""
    if not is_qualified_name(r.key) or any(not is_valid_label_value(v) for v in r.values):
        return None
    has = r.key in labels
    if r.operator == "In":
        return None if not r.values else (has and labels[r.key] in r.values)
    if r.operator == "NotIn":
        return None if not r.values else (not has or labels[r.key] not in r.values)
    if r.operator == "Exists":
        return None if r.values else has
    if r.operator == "DoesNotExist":
        return None if r.values else not has
    if r.operator in ("Gt", "Lt"):
        if len(r.values) != 1 or parse_int64(r.values[0]) is None:
            return None
        if not has:
            return False
        v = parse_int64(labels[r.key])
        if v is None:
            return False
        b = parse_int64(r.values[0])
        return v > b if r.operator == "Gt" else v < b
    return None


def term_match(term, node) -> bool:
    if not term.match_expressions and not term.match_fields:
        return False
    ok = True
    for r in term.match_expressions:
        m = req_match(r, node.labels)
        if m is None:
            return False
        ok = ok and m
    for r in term.match_fields:
        if r.operator not in ("In", "NotIn") or len(r.values) != 1:
            return False
        val = node.name if r.key == "metadata.name" else ""
        m = (val == r.values[0]) if r.operator == "In" else (val != r.values[0])
        ok = ok and m
    return ok


def affinity_ok(pod, node) -> bool:
    if pod.node_selector:
        for k, v in pod.node_selector.items():
            if node.labels.get(k) != v:
                return False
    req = pod.affinity.required_terms if pod.affinity is not None else None
    if req is None:
        return True
    return any(term_match(t, node) for t in req)


def prefilter(pod):
    """NodeAffinity PreFilter: None (all), 'fail', or a set of node names."""
    req = pod.affinity.required_terms if pod.affinity is not None else None
    if not req:
        return None
    union = set()
    for t in req:
        tn = None
        for r in t.match_fields:
            if r.key == "metadata.name" and r.operator == "In":
                tn = set(r.values) if tn is None else tn & set(r.values)
        if tn is None:
            return None
        if not tn:
            return "fail"
        union |= tn
    return union


def ports_of(pod):
    out = []
    for c in pod.containers:
        for p in c.ports:
            if p.host_port > 0:
                out.append((p.host_ip or "0.0.0.0", p.protocol or "TCP", p.host_port))
    return out


def filters(pod, node, node_pods, apply_unsched=True):
    """RunFilterPlugins: the failing plugin's name or None."""
    unsched = Taint("node.kubernetes.io/unschedulable", "", "NoSchedule")
    if apply_unsched and node.unschedulable and not any(tolerates(t, unsched) for t in pod.tolerations):
        return "NodeUnschedulable"
    if pod.node_name and pod.node_name != node.name:
        return "NodeName"
    for t in node.taints:
        if t.effect in ("NoSchedule", "NoExecute") and not any(tolerates(x, t) for x in pod.tolerations):
            return "TaintToleration"
    if (pod.node_selector is not None or (pod.affinity is not None and pod.affinity.required_terms is not None)) \
            and not affinity_ok(pod, node):
        return "NodeAffinity"
    used = set()
    for q in node_pods:
        used |= set(ports_of(q))
    for (ip, proto, port) in ports_of(pod):
        for (ip2, proto2, port2) in used:
            if proto2 == proto and port2 == port and (ip == "0.0.0.0" or ip2 in ("0.0.0.0", ip)):
                return "NodePorts"
    alloc = {k: (_q(v).milli_value() if k == "cpu" else _q(v).value()) for k, v in node.allocatable.items()}
    used_r = {}
    for q in node_pods:
        for k, v in request(q).items():
            used_r[k] = used_r.get(k, 0) + v
    r = request(pod)
    bad = len(node_pods) + 1 > alloc.get("pods", 0)
    scalar_keys = [k for k in r if k not in ("cpu", "memory", "ephemeral-storage")]
    if not (r.get("cpu", 0) == 0 and r.get("memory", 0) == 0 and r.get("ephemeral-storage", 0) == 0
            and not scalar_keys):
        for k in ("cpu", "memory", "ephemeral-storage"):
            if r.get(k, 0) > alloc.get(k, 0) - used_r.get(k, 0):
                bad = True
        for k in scalar_keys:
            if r[k] != 0 and r[k] > alloc.get(k, 0) - used_r.get(k, 0):
                bad = True
    return "NodeResourcesFit" if bad else None
