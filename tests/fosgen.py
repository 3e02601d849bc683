"""Seeded FilterOutSchedulable inputs at the API level: random clusters (randgen) plus
pending pods from controllers with repeated pod specs (similar-pods skips), controllers
with more than 10 pod variants (similar_pods.go:53 cap), DaemonSet pods, priorities and
hints (some naming missing nodes)."""
from __future__ import annotations

import copy
import random

from autoscaler_amd.k8s import OwnerReference, Quantity
from randgen import rand_cluster, rand_pod


def rand_filter_case(seed: int, n_nodes: int = 10, n_pending: int = 60):
    rng, nodes, scheduled, _ = rand_cluster(seed, n_nodes=n_nodes, n_pods=3 * n_nodes)
    pending = []
    k = 0
    while len(pending) < n_pending:
        r = rng.random()
        base = rand_pod(rng, f"q{k}")
        k += 1
        if r < 0.15:                                            # no controller
            base.owner_refs = []
            pending.append(base)
            continue
        kind = "DaemonSet" if r < 0.25 else "ReplicaSet"
        uid = f"{kind}-{k}"
        nvar = rng.randint(11, 14) if rng.random() < 0.2 else rng.randint(1, 3)
        variants = []
        for v in range(nvar):
            pv = rand_pod(rng, f"v{k}-{v}") if v else base
            pv.owner_refs = [OwnerReference(kind, uid, uid)]
            if nvar > 10 and rng.random() < 0.8:                  # a variant that fits nowhere
                pv.containers[0].requests["cpu"] = Quantity.milli(64000 + v)
            if rng.random() < 0.3:
                pv.priority = rng.choice([0, 10, 100])
            variants.append(pv)
        for j in range(rng.randint(15, 30) if nvar > 10 else rng.randint(1, 8)):
            p = copy.deepcopy(rng.choice(variants))
            p.name = f"{p.name}-{j}"
            p.uid = p.name
            pending.append(p)
    pending = pending[:n_pending]
    hints = {}
    for p in pending:
        if rng.random() < 0.25:
            hints[p.uid or f"{p.namespace}/{p.name}"] = rng.choice([n.name for n in nodes] + ["gone"])
    return nodes, scheduled, pending, hints
