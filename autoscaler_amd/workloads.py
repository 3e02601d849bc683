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
from .gosort import sort_slice_desc

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


# ---------------------------------------------------------------------------
# C4: taint / toleration + node-affinity-heavy
# ---------------------------------------------------------------------------
C4_KEYS = 12            # label keys; key 0 is the integer key (Gt/Lt), keys 1..11 string keys
C4_PAIRS = 64           # interned (key, value) pairs over keys 1..11
C4_TAINT_CLASSES = 20


class _C4Universe:
    """Interned attribute universe shared by nodes, templates and pods."""

    def __init__(self, rng):
        # pair p belongs to string key pair_key[p] (1..11), values spread over the keys
        self.pair_key = np.array([1 + (p % (C4_KEYS - 1)) for p in range(C4_PAIRS)], np.int64)
        # taint class effects: 0 NoSchedule, 1 NoExecute, 2 PreferNoSchedule (not a filter)
        self.taint_effect = rng.integers(0, 3, C4_TAINT_CLASSES)
        self.filter_taints = np.nonzero(self.taint_effect != 2)[0]

    def node_attrs(self, rng, n_taints: int):
        """(taint mask, pair bitset word, key mask, int label) of one node / template."""
        classes = rng.choice(C4_TAINT_CLASSES, size=n_taints, replace=False) if n_taints else np.zeros(0, int)
        mask = 0
        for c in classes:
            if self.taint_effect[c] != 2:          # PreferNoSchedule is not interned for filtering
                mask |= 1 << int(c)
        pairs, keys = 0, 1                          # key 0 (integer) always present
        for k in range(1, C4_KEYS):
            if rng.random() < 0.75:
                cand = np.nonzero(self.pair_key == k)[0]
                pairs |= 1 << int(rng.choice(cand))
                keys |= 1 << k
        return mask, pairs, keys, int(rng.integers(0, 100))


def _c4_pod_spec(rng, uni: _C4Universe, terms: list, reqs: list, anchor=None):
    """Tolerations, nodeSelector and required node-affinity terms of one controller's pods.
    anchor = (taints, pairs, keys, ival) of a node the pods must fit (sweep), or None."""
    tol = 0
    if rng.random() < 0.05:
        tol = (1 << 64) - 1                        # a key-less Exists toleration: every taint
    else:
        for c in uni.filter_taints:
            if rng.random() < 0.4:
                tol |= 1 << int(c)
        if anchor is not None:
            tol |= anchor[0]
    sel = 0
    if rng.random() < 0.60:
        if anchor is not None:
            have = [p for p in range(C4_PAIRS) if (anchor[1] >> p) & 1]
            pick = rng.choice(have, size=min(len(have), int(rng.integers(1, 4))), replace=False) if have else []
        else:
            pick = rng.choice(C4_PAIRS, size=int(rng.integers(1, 4)), replace=False)
            # at most one pair per key (a selector with two values of one key matches nothing)
            seen, keep = set(), []
            for p in pick:
                if uni.pair_key[p] not in seen:
                    seen.add(uni.pair_key[p])
                    keep.append(p)
            pick = keep
        for p in pick:
            sel |= 1 << int(p)
    first, count = 0, -1
    if rng.random() < 0.20:
        first, count = len(terms), 2
        for t in range(2):
            tf = len(reqs)
            for e in range(2):
                op = int(rng.choice([abi.CA_OP_IN, abi.CA_OP_NOTIN, abi.CA_OP_EXISTS, abi.CA_OP_GT]))
                r = np.zeros(1, abi.REQ_DTYPE)[0]
                r["op"] = op
                if op == abi.CA_OP_GT:
                    r["key"] = 0
                    r["bound"] = int(rng.integers(0, 60))
                    if anchor is not None and t == 0 and not anchor[3] > r["bound"]:
                        r["bound"] = anchor[3] - 1
                elif op == abi.CA_OP_EXISTS:
                    k = int(rng.integers(1, C4_KEYS))
                    if anchor is not None and t == 0:
                        ks = [kk for kk in range(1, C4_KEYS) if (anchor[2] >> kk) & 1]
                        k = int(rng.choice(ks)) if ks else 0
                    r["key"] = k
                else:
                    k = int(rng.integers(1, C4_KEYS))
                    vals = np.nonzero(uni.pair_key == k)[0]
                    chosen = rng.choice(vals, size=min(len(vals), int(rng.integers(1, 3))), replace=False)
                    word = 0
                    for p in chosen:
                        word |= 1 << int(p)
                    if anchor is not None and t == 0:
                        node_pairs_k = anchor[1] & sum(1 << int(p) for p in vals)
                        if op == abi.CA_OP_IN:
                            word |= node_pairs_k if node_pairs_k else 0
                            if not node_pairs_k:
                                r["op"] = abi.CA_OP_NOTIN
                        else:
                            word &= ~node_pairs_k
                    r["key"] = k
                    r["pairs"][0] = np.uint64(word & ((1 << 64) - 1))
                reqs.append(r)
            terms.append((tf, 2))
    return tol, sel, first, count


def _c4_static_ok(tol, sel, first, count, terms, reqs, node_taints, node_pairs, node_keys, ival) -> bool:
    """Template-side static filters (TaintToleration, NodeAffinity) of one pod spec."""
    if node_taints & ~tol & ((1 << 64) - 1):
        return False
    if (node_pairs & sel) != sel:
        return False
    if count < 0:
        return True
    for t in range(first, first + count):
        tf, tc = terms[t]
        ok = True
        for r in reqs[tf:tf + tc]:
            op, key, bound, word = int(r["op"]), int(r["key"]), int(r["bound"]), int(r["pairs"][0])
            if op == abi.CA_OP_IN:
                ok = (node_pairs & word) != 0
            elif op == abi.CA_OP_NOTIN:
                ok = (node_pairs & word) == 0
            elif op == abi.CA_OP_EXISTS:
                ok = bool((node_keys >> key) & 1)
            elif op == abi.CA_OP_GT:
                ok = ival > bound
            if not ok:
                break
        if ok:
            return True
    return False


def _c4_encode_spec(p, tol, sel, first, count):
    p["tolerated_taints"] = np.uint64(tol & ((1 << 64) - 1))
    p["node_selector"][:, 0] = np.uint64(sel)
    p["aff_term_first"] = first
    p["aff_term_count"] = count
    if sel or count >= 0:
        p["flags"] |= abi.CA_POD_AFFINITY_FILTER


def _c4_node(rec, attrs):
    taints, pairs, keys, ival = attrs
    rec["taints"] = np.uint64(taints)
    rec["label_pairs"][0] = np.uint64(pairs)
    rec["label_keys"] = np.uint64(keys)
    rec["int_label"][0] = ival
    rec["int_label_valid"] = 1


def c4(n_pods: int = 50_000, n_groups: int = 100, n_existing: int = 1000, max_nodes: int = 1000,
       seed: int = 1234, pods_per_controller: int = 100) -> EstimateWorkload:
    """C4 Estimate batch: C2 shapes and templates plus 20 taint classes (0-3 per template),
    64 label pairs over 12 keys (one integer key), 60% of controllers with a nodeSelector of
    1-3 pairs, 20% with 2 required terms x 2 expressions (In/NotIn/Exists/Gt), 5% tolerating
    everything.  Group pod lists = the pods passing CheckPredicates on the template
    (ComputeExpansionOption, orchestrator.go:455-481): resources and static filters."""
    rng = np.random.default_rng(seed)
    uni = _C4Universe(rng)
    shapes = [(c, m) for c in C2_CPU for m in C2_MEM]
    n_ctrl = max(1, (n_pods + pods_per_controller - 1) // pods_per_controller)
    ctrl_shape = rng.integers(0, len(shapes), n_ctrl)
    terms: list = []
    reqs: list = []
    ctrl_spec = [_c4_pod_spec(rng, uni, terms, reqs) for _ in range(n_ctrl)]
    ctrl_of_pod = np.repeat(np.arange(n_ctrl), pods_per_controller)[:n_pods]
    cpu = np.array([shapes[ctrl_shape[c]][0] for c in ctrl_of_pod], np.int64)
    mem = np.array([shapes[ctrl_shape[c]][1] for c in ctrl_of_pod], np.int64)
    pods = resource_pods(cpu, mem)
    pods["similar_class"] = ctrl_of_pod
    for c in range(n_ctrl):
        sl = slice(c * pods_per_controller, min(n_pods, (c + 1) * pods_per_controller))
        _c4_encode_spec(pods[sl], *ctrl_spec[c])
    term_arr = np.array(terms, dtype=abi.TERM_DTYPE) if terms else np.zeros(0, abi.TERM_DTYPE)
    req_arr = np.array(reqs, dtype=abi.REQ_DTYPE) if reqs else np.zeros(0, abi.REQ_DTYPE)
    templates = np.zeros(n_groups, abi.TEMPLATE_DTYPE)
    offs, parts = [0], []
    for g in range(n_groups):
        cores = C2_CORES[rng.integers(0, len(C2_CORES))]
        mpc = C2_MEM_PER_CORE[rng.integers(0, len(C2_MEM_PER_CORE))]
        acpu = cores * 1000 * 95 // 100
        amem = cores * mpc * GI * 95 // 100
        ds = int(rng.integers(0, 4))
        templates[g] = make_template(acpu, amem, 110, ds, name_id=-1000 - g)[0]
        attrs = uni.node_attrs(rng, int(rng.integers(0, 4)))
        _c4_node(templates[g]["node"], attrs)
        free_cpu, free_mem = acpu - ds * 100, amem - ds * 128 * MI
        ok_ctrl = np.array([_c4_static_ok(*ctrl_spec[c], terms, reqs, *attrs) for c in range(n_ctrl)])
        ok = ok_ctrl[ctrl_of_pod] & (cpu <= free_cpu) & (mem <= free_mem)
        sel = np.nonzero(ok)[0].astype(np.int32)
        parts.append(sel)
        offs.append(offs[-1] + len(sel))
    existing = abi.empty_nodes(n_existing)
    existing["alloc_milli_cpu"] = 16000
    existing["alloc_memory"] = 64 * GI
    existing["alloc_pods"] = 110
    existing["name_id"] = np.arange(n_existing)
    for i in range(n_existing):
        _c4_node(existing[i], uni.node_attrs(rng, int(rng.integers(0, 3))))
    pod_idx = np.concatenate(parts).astype(np.int32) if parts else np.zeros(0, np.int32)
    return EstimateWorkload("C4", abi.PodTable(pods, term_arr, req_arr), np.array(offs, np.int32), pod_idx,
                            templates, n_existing, max_nodes, existing,
                            {"seed": seed, "terms": len(term_arr), "reqs": len(req_arr)})


def c4_sweep(n_nodes: int = 5000, pods_per_node: int = 30, seed: int = 4321) -> SweepWorkload:
    """C3 with the C4 attributes: nodes carry 0-2 taint classes and labels, running pods
    tolerate their node's taints (plus random others) and carry selectors / required terms
    their node satisfies, so moving them is restricted by the static filters."""
    w = c3(n_nodes=n_nodes, pods_per_node=pods_per_node, seed=seed)
    rng = np.random.default_rng(seed + 1)
    uni = _C4Universe(rng)
    attrs = [uni.node_attrs(rng, int(rng.integers(0, 3))) for _ in range(n_nodes)]
    for i in range(n_nodes):
        _c4_node(w.nodes[i], attrs[i])
    terms: list = []
    reqs: list = []
    pods = w.table.pods
    # one spec per (node, replica set) group of pods: controllers are per node here
    for i in range(n_nodes):
        for j in range(0, pods_per_node, 10):
            spec = _c4_pod_spec(rng, uni, terms, reqs, anchor=attrs[i])
            sl = slice(i * pods_per_node + j, i * pods_per_node + min(pods_per_node, j + 10))
            _c4_encode_spec(pods[sl], *spec)
    term_arr = np.array(terms, dtype=abi.TERM_DTYPE) if terms else np.zeros(0, abi.TERM_DTYPE)
    req_arr = np.array(reqs, dtype=abi.REQ_DTYPE) if reqs else np.zeros(0, abi.REQ_DTYPE)
    return SweepWorkload("C4-sweep", w.nodes, abi.PodTable(pods, term_arr, req_arr), w.pod_node, w.candidates,
                         w.dest_mask, w.cand_status, w.move_off, w.move_pods,
                         dict(w.meta, seed=seed, terms=len(term_arr)))


# ---------------------------------------------------------------------------
# C5 FilterOutSchedulable: pending pods against a large running cluster
# ---------------------------------------------------------------------------
@dataclass
class FilterWorkload:
    name: str
    nodes: np.ndarray
    table: abi.PodTable          # running pods
    pod_node: np.ndarray
    pending: abi.PodTable        # pending pods
    order: np.ndarray            # priority order (filter_out_schedulable.go:97-99, stable)
    class_owner: np.ndarray      # dense controller id per similar class
    hints: np.ndarray            # hinted node position per order position, -1 none
    meta: dict = field(default_factory=dict)


def c5_filter(n_nodes: int = 15_000, pods_per_node: int = 20, n_pending: int = 20_000, seed: int = 5,
              hint_frac: float = 0.2, taints: bool = False, util_low=(0.70, 0.85),
              util_high=(0.92, 0.99)) -> FilterWorkload:
    """C5's FilterOutSchedulable step: 15k nodes {16 cores, 64Gi, 110
    pods} running 300k pods (30% of nodes at 70-85% cpu, the rest at 92-99%), 20k pending pods
    of C2 shapes from controllers of 50 pods on average; 10% of controllers run 12-20 pod
    variants (past similar_pods' 10-per-controller cache), 3% DaemonSet pods, 5% pods with no
    controller, 4 priority levels, hint_frac of the pods hinted to a random node.
    taints=True adds the C4 taint/label universe to the nodes and the pending pods."""
    rng = np.random.default_rng(seed)
    node_cpu, node_mem = 16000, 64 * GI
    nodes = abi.empty_nodes(n_nodes)
    nodes["alloc_milli_cpu"] = node_cpu
    nodes["alloc_memory"] = node_mem
    nodes["alloc_pods"] = 110
    nodes["name_id"] = np.arange(n_nodes)
    low = rng.random(n_nodes) < 0.30
    util = np.where(low, rng.uniform(*util_low, n_nodes), rng.uniform(*util_high, n_nodes))
    w = rng.gamma(2.0, 1.0, (n_nodes, pods_per_node))
    w /= w.sum(axis=1, keepdims=True)
    cpu = np.floor(w * (util * node_cpu)[:, None]).astype(np.int64).ravel()
    mem = (np.floor(w * (util * node_mem / MI)[:, None]).astype(np.int64) * MI).ravel()
    running = resource_pods(cpu, mem)
    pod_node = np.repeat(np.arange(n_nodes, dtype=np.int32), pods_per_node)
    # pending pods: controllers -> variants (similar classes) -> pods
    shapes = [(c, m) for c in C2_CPU for m in C2_MEM]
    cls_shape, cls_owner, cls_ds = [], [], []
    pod_cls = []
    n_owner = 0
    while len(pod_cls) < n_pending:
        r = rng.random()
        if r < 0.05:                                   # no controller: class -1
            pod_cls.extend([-1] * int(rng.integers(1, 4)))
            continue
        ds = r < 0.08
        nvar = int(rng.integers(12, 21)) if (not ds and rng.random() < 0.10) else 1
        first = len(cls_shape)
        for _ in range(nvar):
            cls_shape.append(int(rng.integers(0, len(shapes))))
            cls_owner.append(n_owner)
            cls_ds.append(ds)
        n_owner += 1
        npods = int(rng.integers(1, 100))
        pod_cls.extend((first + rng.integers(0, nvar, npods)).tolist())
    pod_cls = np.array(pod_cls[:n_pending], np.int64)
    noc = pod_cls < 0
    free_shape = rng.integers(0, len(shapes), n_pending)
    shp = np.where(noc, free_shape, np.array(cls_shape + [0], np.int64)[pod_cls])
    pcpu = np.array([shapes[s][0] for s in shp], np.int64)
    pmem = np.array([shapes[s][1] for s in shp], np.int64)
    pend = resource_pods(pcpu, pmem)
    pend["similar_class"] = pod_cls
    ds_pod = np.array(cls_ds + [False])[pod_cls] & ~noc
    pend["flags"][ds_pod] |= abi.CA_POD_DAEMONSET
    terms_arr = req_arr = None
    if taints:
        uni = _C4Universe(rng)
        for i in range(n_nodes):
            _c4_node(nodes[i], uni.node_attrs(rng, int(rng.integers(0, 3))))
        terms: list = []
        reqs: list = []
        n_cls = len(cls_shape)
        specs = [_c4_pod_spec(rng, uni, terms, reqs) for _ in range(n_cls + 1)]
        for i in range(n_pending):
            c = int(pod_cls[i])
            if c < 0:                                  # a pod of its own: its own spec
                _c4_encode_spec(pend[i:i + 1], *_c4_pod_spec(rng, uni, terms, reqs))
            else:
                _c4_encode_spec(pend[i:i + 1], *specs[c])
        terms_arr = np.array(terms, dtype=abi.TERM_DTYPE) if terms else np.zeros(0, abi.TERM_DTYPE)
        req_arr = np.array(reqs, dtype=abi.REQ_DTYPE) if reqs else np.zeros(0, abi.REQ_DTYPE)
    prio = rng.choice([0, 100, 1000, 10000], n_pending, p=[0.6, 0.2, 0.15, 0.05])
    # a class's pods share their spec, priority included
    cls_prio = rng.choice([0, 100, 1000, 10000], len(cls_shape) + 1, p=[0.6, 0.2, 0.15, 0.05])
    prio = np.where(noc, prio, cls_prio[pod_cls])
    # filterOutSchedulableByPacking's sort.Slice by priority, descending
    # (filter_out_schedulable.go:97-99): Go 1.19's pdqsort order, ties included
    order = np.array(sort_slice_desc(prio.tolist()), np.int32)
    hints = np.where(rng.random(n_pending) < hint_frac, rng.integers(0, n_nodes, n_pending), -1).astype(np.int32)
    pending = abi.PodTable(pend, terms_arr, req_arr) if taints else abi.PodTable(pend)
    return FilterWorkload("C5-filter" + ("-c4" if taints else ""), nodes, abi.PodTable(running), pod_node, pending,
                          order, np.array(cls_owner, np.int32), hints,
                          {"seed": seed, "classes": len(cls_shape), "controllers": n_owner,
                           "daemonset_pods": int(ds_pod.sum()), "no_controller_pods": int(noc.sum())})


def load_filter(backend, w: FilterWorkload) -> None:
    backend.clear()
    backend.add_nodes(w.nodes)
    backend.add_pods(w.table, np.arange(len(w.table), dtype=np.int32), w.pod_node)


def util_table(seed: int = 11, n_nodes: int = 15000, pods_per_node: int = 20, now_ns: int = 1_608_310_800 * 10**9,
               edge_cases: bool = True):
    """Scale-down eligibility input at C5 size by default: ca_util_node /
    ca_util_pod rows with a ragged pod count per node (0 .. 2 x pods_per_node), 5% DaemonSet,
    2% mirror, 3% deleted pods whose deletion lands either side of the long-terminating
    cut-off, ~10% GPU-config nodes, and (edge_cases) nodes with missing or zero
    allocatable and DaemonSet shares equal to allocatable (x/0 -> inf/nan).
    Returns (nodes, pod_off, pods, now_ns)."""
    from . import abi
    rng = np.random.default_rng(seed)
    counts = rng.integers(0, 2 * pods_per_node + 1, n_nodes)
    pod_off = np.zeros(n_nodes + 1, np.int32)
    np.cumsum(counts, out=pod_off[1:])
    P = int(pod_off[-1])
    nodes = np.zeros(n_nodes, abi.UTIL_NODE_DTYPE)
    nodes["alloc_milli"][:, 0] = rng.choice([4000, 8000, 16000, 32000], n_nodes)
    nodes["alloc_milli"][:, 1] = rng.choice([16, 32, 64, 128], n_nodes) * (1 << 30) * 1000
    nodes["alloc_milli"][:, 2] = rng.choice([1, 2, 4, 8], n_nodes) * 1000
    flags = np.full(n_nodes, abi.CA_UNODE_HAS_CPU | abi.CA_UNODE_HAS_MEM, np.uint32)
    gpu = rng.random(n_nodes) < 0.1
    flags[gpu] |= abi.CA_UNODE_GPU_CONFIG | abi.CA_UNODE_HAS_GPU
    pods = np.zeros(P, abi.UTIL_POD_DTYPE)
    pods["req_milli"][:, 0] = rng.choice([50, 100, 250, 500, 1000], P)
    pods["req_milli"][:, 1] = rng.choice([64, 128, 256, 512, 1024, 2048], P) * (1 << 20) * 1000
    pods["req_milli"][:, 2] = (rng.random(P) < 0.3) * 1000
    u = rng.random(P)
    pf = np.zeros(P, np.uint32)
    pf[u < 0.05] |= abi.CA_UPOD_DAEMONSET
    pf[(u >= 0.05) & (u < 0.07)] |= abi.CA_UPOD_MIRROR
    dele = (u >= 0.07) & (u < 0.10)
    pf[dele] |= abi.CA_UPOD_DELETED
    pods["grace_s"][dele] = rng.choice([0, 30, 600], int(dele.sum()))
    pods["deletion_ns"][dele] = now_ns - rng.integers(0, 1200, int(dele.sum())) * 10**9
    d = rng.random(P)
    pf[d < 0.6] |= abi.CA_UPOD_MOVABLE
    pf[d > 0.98] |= abi.CA_UPOD_BLOCKING
    if edge_cases and n_nodes >= 64:
        e = rng.choice(n_nodes, 48, replace=False)
        flags[e[0:8]] &= ~np.uint32(abi.CA_UNODE_HAS_CPU)
        nodes["alloc_milli"][e[8:16], 0] = 0
        flags[e[16:24]] &= ~np.uint32(abi.CA_UNODE_HAS_MEM)
        nodes["alloc_milli"][e[24:32], 1] = 0
        flags[e[32:40]] &= ~np.uint32(abi.CA_UNODE_HAS_GPU)       # unready GPU (label, no allocatable)
        flags[e[32:40]] |= abi.CA_UNODE_GPU_CONFIG
        for n in e[40:48]:                                         # DaemonSets use the whole node
            b, f = pod_off[n], pod_off[n + 1]
            if f > b:
                pf[b:f] = abi.CA_UPOD_DAEMONSET
                pods["req_milli"][b, :] = nodes["alloc_milli"][n, :]
                pods["req_milli"][b + 1:f, :] = 0
        empty = e[40:48]
        for n in empty[:4]:
            pf[pod_off[n]:pod_off[n + 1]] &= ~np.uint32(abi.CA_UPOD_MOVABLE | abi.CA_UPOD_BLOCKING)
    nodes["flags"] = flags
    pods["flags"] = pf
    return nodes, pod_off, pods, now_ns
