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


# Shapes whose float64 scores tie ACROSS shapes on a 4000m / 16Gi template (and on its
# multiples): c / 4000 + m / 16Gi is 0.3125 for the first three, 0.5 for the next three,
# 0.8125 for the pair after; the last three tie with nothing.
TIE_SHAPES = [(1000, 1 << 30), (500, 3 << 30), (250, 4 << 30),
              (1500, 2 << 30), (1000, 4 << 30), (500, 6 << 30),
              (750, 10 << 30), (2000, 5 << 30),
              (100, 128 << 20), (300, 700 << 20), (1200, 1536 << 20)]


def tied_workload(seed, n_pods=6000, n_groups=8):
    """An Estimate batch of uniform score classes (pods identical but for their controller)
    with cross-class float64 score ties on most templates, controllers interleaved in short
    runs so Go's pdqsort mixes the tied classes.  Returns (workload, shape of every pod)."""
    from autoscaler_amd import workloads as W
    rng = np.random.default_rng(1000 + seed)
    per_ctrl = int(rng.integers(3, 9))
    n_ctrl = (n_pods + per_ctrl - 1) // per_ctrl
    ctrl_shape = rng.integers(0, len(TIE_SHAPES), n_ctrl)
    shape_of = np.repeat(ctrl_shape, per_ctrl)[:n_pods].astype(np.int64)
    cpu = np.array([TIE_SHAPES[s][0] for s in shape_of], np.int64)
    mem = np.array([TIE_SHAPES[s][1] for s in shape_of], np.int64)
    pods = W.resource_pods(cpu, mem)
    pods["similar_class"] = np.repeat(np.arange(n_ctrl), per_ctrl)[:n_pods]
    templates = np.zeros(n_groups, abi.TEMPLATE_DTYPE)
    offs, parts = [0], []
    for g in range(n_groups):
        k = (1, 2, 4, 1, 3)[g % 5]                         # 3 x 4000m: 1200m / 48Gi-score ties too
        acpu, amem = 4000 * k, (16 << 30) * k
        if g % 5 == 3:
            acpu, amem = 6000, 20 << 30                    # a template without ties
        ds = int(rng.integers(0, 3))
        templates[g] = W.make_template(acpu, amem, 110, ds, name_id=-1000 - g)[0]
        ok = (cpu <= acpu - ds * 100) & (mem <= amem - ds * 128 * W.MI)
        sel = np.nonzero(ok & (rng.random(n_pods) < 0.8))[0].astype(np.int32)
        parts.append(sel)
        offs.append(offs[-1] + len(sel))
    n_existing = (0, 20, 200)[seed % 3]
    existing = abi.empty_nodes(n_existing)
    existing["alloc_milli_cpu"] = 8000
    existing["alloc_memory"] = 32 << 30
    existing["alloc_pods"] = 110
    existing["name_id"] = np.arange(n_existing)
    w = W.EstimateWorkload("C2-ties", abi.PodTable(pods), np.array(offs, np.int32), np.concatenate(parts),
                           templates, n_existing, (1000, 0, 9)[seed % 3], existing, {"seed": seed})
    return w, shape_of
