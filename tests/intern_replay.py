"""The interning calls a cgo shim makes through casim.h "interning", in the order
autoscaler_amd/intern.py interns (Interner.observe, then encode_nodes, then encode_pods), over
API objects (autoscaler_amd/k8s.py).  Drives any object with the ca_intern_* method set:
``native.CInterner`` (tests/test_intern_c.py compares it with intern.py) or the recorder of
tests/golden/make_intern_calls.py (which writes the calls with intern_fixtures.json's
expectations for tests/c_abi/intern_driver.c).  Test infrastructure."""
from autoscaler_amd.intern import pod_ports


def _terms(p):
    return p.affinity.required_terms if (p.affinity is not None and p.affinity.required_terms) else []


def _term_reqs(term):
    return ([(r.key, r.operator, list(r.values), False) for r in term.match_expressions]
            + [(r.key, r.operator, list(r.values), True) for r in term.match_fields])


def replay(api, nodes, pods, tmpls=()):
    """api methods: taint, label_pair, label_key, int_key, port, resource, name (-> id),
    is_scalar(name) -> bool, encode_node(i, labels, taints), encode_pod(i, tols, ports,
    selector, terms) where terms is a list of requirement lists (non-empty terms only)."""
    tnodes = [t[0] for t in tmpls]
    tpods = [p for t in tmpls for p in t[1]]
    # observe (intern.py:Interner.observe)
    for n in list(nodes) + tnodes:
        api.name(n.name)
        for t in n.taints:
            api.taint(t.key, t.value, t.effect)
        for r in n.allocatable:
            api.resource(r)
    for p in list(pods) + tpods:
        for c in p.containers + p.init_containers:
            for r in c.requests:
                api.resource(r)
        for r in (p.overhead or {}):
            api.resource(r)
        for k, v in (p.node_selector or {}).items():
            api.label_pair(k, v)
        for term in _terms(p):
            for r in term.match_expressions:
                if r.operator in ("In", "NotIn"):
                    for v in r.values:
                        api.label_pair(r.key, v)
                elif r.operator in ("Exists", "DoesNotExist"):
                    api.label_key(r.key)
                elif r.operator in ("Gt", "Lt"):
                    api.int_key(r.key)
        for ip, proto, port in pod_ports(p):
            api.port(ip, proto, port)
        if p.node_name:
            api.name(p.node_name)
    # encode_nodes
    for i, n in enumerate(nodes):
        api.encode_node(i, dict(n.labels), [(t.key, t.value, t.effect) for t in n.taints])
    # encode_pods (tolerations, ports, node name, selector, terms, PreFilter names: _encode_pod's order)
    for i, p in enumerate(pods):
        tols = [(t.key, t.operator, t.value, t.effect) for t in p.tolerations]
        required = p.affinity.required_terms if p.affinity is not None else None
        terms = [_term_reqs(t) for t in (required or []) if (t.match_expressions or t.match_fields)]
        api.encode_pod(i, tols, pod_ports(p), p.node_name, dict(p.node_selector or {}), terms,
                       _prefilter_names(required))


def _prefilter_names(required):
    """NodeAffinity.PreFilter NodeNames (node_affinity.go:106-135) as intern.py computes
    them: the names the shim interns after the terms (sorted), [] for none / all nodes."""
    if not required:
        return []
    union = None
    for term in required:
        tn = None
        for r in term.match_fields:
            if r.key == "metadata.name" and r.operator == "In":
                s = set(r.values)
                tn = s if tn is None else tn & s
        if tn is None or not tn:
            return []
        union = tn if union is None else union | tn
    return sorted(union)
