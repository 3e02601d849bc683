"""Seeded synthetic clusters for the BASELINE.json configurations.

Each generator returns ABI records (numpy arrays of the casim.h dtypes) so the
same inputs feed the HIP path and the CPU restatement.  Sizes are parameters so
the parity tests can run scaled-down copies of the bench workloads.

  C1  1k identical pods {500m, 1Gi} -> template {4000m, 16Gi, 110 pods}  (125 nodes)
  C2  50k heterogeneous pods (64-shape catalog) x 100 node-group templates,
      N = 1000 existing nodes, resource-fit only
  C3  5k-node / 150k-pod scale-down sweep (legacy FindNodesToRemove)
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import abi

MI = 1024 * 1024
GI = 1024 * MI


@dataclass
class EstimateWorkload:
    name: str
    table: abi.PodTable
    group_off: np.ndarray
    pod_idx: np.ndarray
    templates: np.ndarray
    n_existing: int
    max_nodes: int
    existing_nodes: np.ndarray
    meta: dict = field(default_factory=dict)


@dataclass
class SweepWorkload:
    name: str
    nodes: np.ndarray
    table: abi.PodTable          # scheduled pods (one record each)
    pod_node: np.ndarray         # node position of every pod
    candidates: np.ndarray
    dest_mask: np.ndarray
    cand_status: np.ndarray
    move_off: np.ndarray
    move_pods: np.ndarray        # indices into table == mirror pod ids (pods added in order)
    meta: dict = field(default_factory=dict)


def make_node(cpu_milli: int, mem: int, pods: int = 110, name_id: int = 0, eph: int = 0) -> np.ndarray:
    n = abi.empty_nodes(1)
    n["alloc_milli_cpu"] = cpu_milli
    n["alloc_memory"] = mem
    n["alloc_ephemeral"] = eph
    n["alloc_pods"] = pods
    n["name_id"] = name_id
    return n


def make_template(cpu_milli: int, mem: int, pods: int = 110, ds_pods: int = 0, ds_cpu: int = 100,
                  ds_mem: int = 128 * MI, name_id: int = -1000) -> np.ndarray:
    t = np.zeros(1, abi.TEMPLATE_DTYPE)
    t["node"] = make_node(cpu_milli, mem, pods, name_id)
    t["used_milli_cpu"] = ds_pods * ds_cpu
    t["used_memory"] = ds_pods * ds_mem
    t["used_pods"] = ds_pods
    return t


def resource_pods(cpu: np.ndarray, mem: np.ndarray) -> np.ndarray:
    """Single-container pods requesting (cpu milli, mem bytes); containers-only sums == requests."""
    p = abi.empty_pods(len(cpu))
    p["req_milli_cpu"] = cpu
    p["req_memory"] = mem
    p["score_milli_cpu"] = cpu
    p["score_memory"] = mem
    return p


# ---------------------------------------------------------------------------
# C1
# ---------------------------------------------------------------------------
def c1(n_pods: int = 1000) -> EstimateWorkload:
    pods = resource_pods(np.full(n_pods, 500), np.full(n_pods, GI))
    tmpl = make_template(4000, 16 * GI, 110)
    return EstimateWorkload("C1", abi.PodTable(pods), np.array([0, n_pods], np.int32),
                            np.arange(n_pods, dtype=np.int32), tmpl, 0, 0, abi.empty_nodes(0),
                            {"expected_nodes": n_pods // 8})


# ---------------------------------------------------------------------------
# C2
# ---------------------------------------------------------------------------
C2_CPU = [100, 250, 500, 750, 1000, 1500, 2000, 4000]
C2_MEM = [128 * MI * (2 ** i) for i in range(8)]          # 128Mi .. 16Gi
C2_CORES = [2, 4, 8, 16, 32, 48, 64, 96]
C2_MEM_PER_CORE = [2, 4, 8]


def c2(n_pods: int = 50_000, n_groups: int = 100, n_existing: int = 1000, max_nodes: int = 1000,
       seed: int = 42, pods_per_controller: int = 100, n_random_shapes: int = 0) -> EstimateWorkload:
    """C2.  n_random_shapes > 0 replaces the 64-shape catalog by that many
    random (cpu, mem) shapes (test variant: many score classes, cross-shape ties allowed)."""
    rng = np.random.default_rng(seed)
    shapes = [(c, m) for c in C2_CPU for m in C2_MEM]
    if n_random_shapes > 0:
        shapes = list({(int(c), int(m) * MI) for c, m in zip(rng.integers(1, 8000, n_random_shapes),
                                                                rng.integers(1, 32768, n_random_shapes))})
    n_ctrl = max(1, (n_pods + pods_per_controller - 1) // pods_per_controller)
    ctrl_shape = rng.integers(0, len(shapes), n_ctrl)
    shape_of_pod = np.repeat(ctrl_shape, pods_per_controller)[:n_pods]
    cpu = np.array([shapes[s][0] for s in shape_of_pod], np.int64)
    mem = np.array([shapes[s][1] for s in shape_of_pod], np.int64)
    pods = resource_pods(cpu, mem)
    pods["similar_class"] = np.repeat(np.arange(n_ctrl), pods_per_controller)[:n_pods]
    templates = np.zeros(n_groups, abi.TEMPLATE_DTYPE)
    offs = [0]
    idx_parts = []
    ties = 0
    for g in range(n_groups):
        cores = C2_CORES[rng.integers(0, len(C2_CORES))]
        mpc = C2_MEM_PER_CORE[rng.integers(0, len(C2_MEM_PER_CORE))]
        acpu = cores * 1000 * 95 // 100
        amem = cores * mpc * GI * 95 // 100
        ds = int(rng.integers(0, 4))
        templates[g] = make_template(acpu, amem, 110, ds, name_id=-1000 - g)[0]
        free_cpu, free_mem = acpu - ds * 100, amem - ds * 128 * MI
        # ComputeExpansionOption: equivalence groups passing CheckPredicates on the template
        ok = (cpu <= free_cpu) & (mem <= free_mem)
        sel = np.nonzero(ok)[0].astype(np.int32)
        idx_parts.append(sel)
        offs.append(offs[-1] + len(sel))
        # H2 check: distinct shapes tying in float64 score for this template
        sc = {}
        if n_random_shapes <= 0:
            for (c, m) in shapes:
                s = c / acpu + m / amem
                sc.setdefault(s, set()).add((c, m))
            ties += sum(1 for v in sc.values() if len(v) > 1)
    pod_idx = np.concatenate(idx_parts) if idx_parts else np.zeros(0, np.int32)
    existing = abi.empty_nodes(n_existing)
    existing["alloc_milli_cpu"] = 16000
    existing["alloc_memory"] = 64 * GI
    existing["alloc_pods"] = 110
    existing["name_id"] = np.arange(n_existing)
    return EstimateWorkload("C2", abi.PodTable(pods), np.array(offs, np.int32), pod_idx.astype(np.int32),
                            templates, n_existing, max_nodes, existing,
                            {"seed": seed, "cross_shape_score_ties": ties})


# ---------------------------------------------------------------------------
# C3
# ---------------------------------------------------------------------------
def c3(n_nodes: int = 5000, pods_per_node: int = 30, seed: int = 7, n_rs: int = 500,
       ds_frac: float = 0.05, unrepl_frac: float = 0.01, kube_system_frac: float = 0.01) -> SweepWorkload:
    rng = np.random.default_rng(seed)
    node_cpu, node_mem = 16000, 64 * GI
    nodes = abi.empty_nodes(n_nodes)
    nodes["alloc_milli_cpu"] = node_cpu
    nodes["alloc_memory"] = node_mem
    nodes["alloc_pods"] = 110
    nodes["name_id"] = np.arange(n_nodes)
    low = rng.random(n_nodes) < 0.30
    util = np.where(low, rng.uniform(0.20, 0.40, n_nodes), rng.uniform(0.60, 0.95, n_nodes))
    P = n_nodes * pods_per_node
    # split each node's cpu/mem budget over its pods (Dirichlet-like weights)
    w = rng.gamma(2.0, 1.0, (n_nodes, pods_per_node))
    w /= w.sum(axis=1, keepdims=True)
    cpu = np.floor(w * (util * node_cpu)[:, None]).astype(np.int64).ravel()
    wm = rng.gamma(2.0, 1.0, (n_nodes, pods_per_node))
    wm /= wm.sum(axis=1, keepdims=True)
    mutil = np.clip(util * rng.uniform(0.7, 1.1, n_nodes), 0.05, 0.98)
    mem = (np.floor(wm * (mutil * node_mem / MI)[:, None]).astype(np.int64) * MI).ravel()
    pods = resource_pods(cpu, mem)
    kind = rng.random(P)
    is_ds = kind < ds_frac
    is_unrepl = (kind >= ds_frac) & (kind < ds_frac + unrepl_frac)
    is_ks = (kind >= ds_frac + unrepl_frac) & (kind < ds_frac + unrepl_frac + kube_system_frac)
    pods["flags"][is_ds] |= abi.CA_POD_DAEMONSET
    rs = rng.integers(0, n_rs, P)
    pods["similar_class"] = np.where(is_ds, -1, rs)
    pod_node = np.repeat(np.arange(n_nodes, dtype=np.int32), pods_per_node)
    # host-side drain verdict per candidate (GetPodsToMove, drain.go:50-90)
    blocked = np.zeros(n_nodes, bool)
    np.logical_or.at(blocked, pod_node, is_unrepl | is_ks)
    cand_status = np.where(blocked, abi.CA_UNREMOVABLE_BLOCKED_BY_POD, 0).astype(np.int32)
    movable = ~is_ds
    move_off = np.zeros(n_nodes + 1, np.int32)
    counts = np.bincount(pod_node[movable], minlength=n_nodes)
    counts[blocked] = 0
    move_off[1:] = np.cumsum(counts)
    keep = movable & ~blocked[pod_node]
    move_pods = np.nonzero(keep)[0].astype(np.int32)       # pods are added node by node, in order
    return SweepWorkload("C3", nodes, abi.PodTable(pods), pod_node, np.arange(n_nodes, dtype=np.int32),
                         np.ones(n_nodes, np.uint8), cand_status, move_off, move_pods,
                         {"seed": seed, "blocked": int(blocked.sum()), "moves": int(len(move_pods))})


def load_estimate(backend, w: EstimateWorkload) -> None:
    backend.clear()
    if len(w.existing_nodes):
        backend.add_nodes(w.existing_nodes)


def load_sweep(backend, w: SweepWorkload) -> np.ndarray:
    backend.clear()
    backend.add_nodes(w.nodes)
    ids = backend.add_pods(w.table, np.arange(len(w.table), dtype=np.int32), w.pod_node)
    return ids
