"""Random Estimate inputs (API objects -> interned ABI records) shared by the GPU parity
tests and the CPU multi-rank tests."""
import random

import numpy as np

from autoscaler_amd import abi
from autoscaler_amd.intern import Interner
from randgen import rand_node, rand_pod


def _estimate_inputs(seed, n_groups=6, n_pods=80):
    rng = random.Random(seed)
    nodes = [rand_node(rng, f"e{i}") for i in range(rng.randint(0, 5))]
    pods = [rand_pod(rng, f"q{i}", small=rng.random() < 0.5) for i in range(n_pods)]
    for p in pods:            # Estimate inputs never carry nodeName / matchFields in these runs
        p.node_name = ""
        if p.affinity is not None and p.affinity.required_terms:
            for t in p.affinity.required_terms:
                t.match_fields = []
    templates = []
    for g in range(n_groups):
        t = rand_node(rng, f"tmpl{g}", big=rng.random() < 0.5)
        ds = [rand_pod(rng, f"ds{g}-{j}", small=True) for j in range(rng.randint(0, 2))]
        for d in ds:
            d.affinity = None
            d.node_selector = None
        templates.append((t, ds))
    groups = []
    for g in range(n_groups):
        sel = [p for p in pods if rng.random() < 0.6]
        groups.append(sel)
    return rng, nodes, pods, templates, groups


def _encode_estimate(nodes, pods, templates, groups):
    it = Interner(nodes, pods, templates)
    table = it.encode_pods(pods)
    node_recs = it.encode_nodes(nodes)
    tm = np.zeros(len(templates), abi.TEMPLATE_DTYPE)
    for g, (t, ds) in enumerate(templates):
        tm[g] = it.encode_template(t, ds)
    idx = {id(p): i for i, p in enumerate(pods)}
    off = [0]
    pod_idx = []
    for sel in groups:
        pod_idx.extend(idx[id(p)] for p in sel)
        off.append(len(pod_idx))
    return table, node_recs, tm, np.array(off, np.int32), np.array(pod_idx, np.int32)
