"""RunOnce's simulation legs at C5 scale, end to end.

One autoscaler loop over a 15k-node / 300k-pod cluster with 20k pending pods, in the
order CA/core/static_autoscaler.go runs them, every step through the kernels' interface on
one backend — the HIP mirror (``native.Mirror`` + ``native.UtilTable``), or the CPU
restatement (``pyoracle``) for parity and the CPU baseline:

1. **FilterOutSchedulable** (static_autoscaler.go:528 → podlistprocessor
   filter_out_schedulable.go:95-124): the pending pods that fit existing nodes are added to
   the snapshot; the rest stay unschedulable.
2. **Expansion options** (static_autoscaler.go:576 → ScaleUp, orchestrator.go:455-481):
   pod equivalence groups of the unschedulable pods (here: one per controller variant,
   ``similar_class``; pods without a controller are their own group), CheckPredicates of
   each group's sample pod on a fresh copy of every node group's template
   (``check_templates``); an option's pods are the groups that pass.
3. **Estimate** of every option (orchestrator.go:139-178, binpacking_estimator.go:65-159),
   one batch, the limiter at 1000 nodes.
4. **Scale-down eligibility** (static_autoscaler.go:615 → legacy.go UpdateUnneededNodes):
   utilization.Calculate of every node (info.go:48-127) over the snapshot after step 1;
   candidates are the nodes below ScaleDownUtilizationThreshold (0.5); the empty ones
   are FindEmptyNodesToRemove's (cluster.go:187-202).
5. **FindNodesToRemove** (cluster.go:116-254) over the non-empty candidates, every node a
   destination, all pods movable (the synthetic pods are ReplicaSet-owned), fresh hints.

The host glue (grouping, building the utilization rows from the snapshot) is numpy and
identical for both backends; each step's device call is timed on its own.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np

from . import abi
from . import workloads as W

UTIL_THRESHOLD = 0.5           # --scale-down-utilization-threshold default (main.go)
MAX_NODES = 1000               # --max-nodes-per-scaleup default


@dataclass
class RunOnceWorkload:
    filt: W.FilterWorkload     # cluster + pending pods (C5)
    templates: np.ndarray      # node groups (TEMPLATE_DTYPE)
    now_ns: int = 1_608_310_800 * 10**9


@dataclass
class RunOnceResult:
    filter_node: np.ndarray = None
    filter_evals: int = 0
    last_index: int = 0
    options: np.ndarray = None           # [G][E] uint8: equivalence group e fits node group g
    est_results: np.ndarray = None
    est_sched: np.ndarray = None
    util: np.ndarray = None
    candidates: np.ndarray = None
    empty: np.ndarray = None
    sweep_results: np.ndarray = None
    sweep_dest: np.ndarray = None
    sweep_hints: np.ndarray = None       # hints of the moved pods, in move order (pod ids differ per backend)
    ms: dict = field(default_factory=dict)
    sizes: dict = field(default_factory=dict)


def c5_runonce(seed: int = 5, n_nodes: int = 15_000, n_pending: int = 20_000, n_groups: int = 100,
               low_frac_util=(0.10, 0.45)) -> RunOnceWorkload:
    """C5: c5_filter's cluster with 30% of the nodes lightly used (scale-down
    candidates) and the rest at 70-99%, its 20k pending pods, and C2's 100 node-group
    templates."""
    import dataclasses
    f = W.c5_filter(n_nodes=n_nodes, n_pending=n_pending, seed=seed, util_low=low_frac_util,
                    util_high=(0.70, 0.99))
    # 15% of the controller variants ask for more than an existing 16-core node has (20 or
    # 28 cores): they stay unschedulable and drive the scale-up legs, as in a real backlog
    rng = np.random.default_rng(seed + 1)
    pods = f.pending.pods.copy()
    big_cls = np.nonzero(rng.random(f.meta["classes"]) < 0.15)[0]
    big = np.isin(pods["similar_class"], big_cls) & (pods["similar_class"] >= 0)
    cores = np.where(rng.random(len(pods)) < 0.5, 20000, 28000)
    for k in ("req_milli_cpu", "score_milli_cpu"):
        pods[k] = np.where(big, cores[pods["similar_class"].clip(0) % len(cores)], pods[k])
    f = dataclasses.replace(f, pending=abi.PodTable(pods))
    t = W.c2(n_pods=1, n_groups=n_groups, n_existing=0).templates
    return RunOnceWorkload(f, t)


def _equivalence_groups(pods: np.ndarray, unsched: np.ndarray):
    """BuildPodGroups (equivalence/groups.go:38-102) restricted to what the synthetic pods
    carry: pods of one controller variant (similar class) are equivalent; a pod without one
    is a group of its own.  First-occurrence order (Go ranges over a map: H2-style order)."""
    cls = pods["similar_class"][unsched]
    groups, where = [], {}
    for k, (i, c) in enumerate(zip(unsched.tolist(), cls.tolist())):
        if c < 0:
            groups.append([i])
            continue
        g = where.get(c)
        if g is None:
            where[c] = len(groups)
            groups.append([i])
        else:
            groups[g].append(i)
    return groups


def _zeros(key: str, n: int, dtype) -> np.ndarray:
    return np.zeros(n, dtype)


class DeviceUtil:
    """The device's utilization step: one resident ca_util_table per loop start snapshot,
    the pods FilterOutSchedulable added sent as ca_util_table_set_added.

    The rows it returns are views into two page-locked buffers used in turn: the result of
    call k is overwritten by call k + 2.  A caller that keeps ``RunOnceResult.util`` across
    loops copies it (``np.copy``) first.  (The CPU port's utilization step for parity and
    the baseline is ``pyoracle.runonce_cpu_util``, outside the package.)"""
    want = "added"

    def __init__(self, device: int = 0):
        self.device = device
        self.table = None
        self.base = None
        self.rows = None                 # page-locked result rows (native.PinnedRows), two in turn:
        self.turn = 0                    # a result stays valid until the call after the next
        self.inputs = None               # page-locked added-pod arrays (UtilInput builds them)

    def zeros(self, key: str, n: int, dtype) -> np.ndarray:
        """Allocator of the loop's added-pod arrays: page-locked, so set_added copies them in
        place (valid until the next loop's UtilInput)."""
        from . import native
        self.inputs = self.inputs or native.PinnedRows()
        return self.inputs.zeros(key, n, dtype)

    def __call__(self, ui: "UtilInput", now_ns: int):
        from . import native
        if self.table is None or self.base is not ui.base:
            if self.table is not None:
                self.table.close()
            self.table = native.UtilTable(self.device, *ui.base)
            self.base = ui.base
            self.rows = self.rows or native.PinnedRows()
            for k in (0, 1):             # both result buffers allocated and touched up front
                self.rows.zeros(f"info{k}", len(ui.base[0]), abi.UTIL_INFO_DTYPE)
        self.table.set_added(ui.added_node, ui.added_pods)
        self.turn ^= 1
        out = self.rows.zeros(f"info{self.turn}", len(ui.base[0]), abi.UTIL_INFO_DTYPE, zero=False)   # all rows written
        return self.table.calculate(False, False, now_ns, out=out)

    def close(self):
        if self.table is not None:
            self.table.close()
            self.table = None
        for r in (self.rows, self.inputs):
            if r is not None:
                r.close()
        self.rows = self.inputs = None


class DeviceExpansion:
    """The device's expansion-option step: the node groups' templates resident in one
    ca_expansion_plan (re-created when the caller's templates change, in place or not), the
    results written by the kernel into a page-locked buffer.  Like DeviceUtil's rows, the
    returned array is overwritten by the next call."""

    def __init__(self):
        self.plan = None
        self.templates = None
        self.tbytes = None
        self.rows = None

    def __call__(self, backend, podset, samples: np.ndarray, templates: np.ndarray) -> np.ndarray:
        from . import native
        # the resident rows are re-uploaded when the node groups change: a new array, or the
        # same array updated in place (keyed on the content, not only the identity)
        tb = np.ascontiguousarray(templates).tobytes()
        if self.plan is None or self.templates is not templates or self.tbytes != tb or self.plan.mirror is not backend:
            if self.plan is not None:
                self.plan.close()
            self.plan = native.ExpansionPlan(backend, templates)
            self.templates = templates
            self.tbytes = tb
            self.rows = self.rows or native.PinnedRows()
        # the loop needs only the option set: one verdict byte per (group, sample) crosses PCIe
        # instead of a 16-byte ca_pred_result
        out = self.rows.zeros("ok", len(templates) * len(samples), np.uint8, zero=False)
        return self.plan.run(podset, samples, verdict_only=True, out=out.reshape(len(templates), len(samples)))

    def close(self):
        if self.plan is not None:
            self.plan.close()
            self.plan = None
        if self.rows is not None:
            self.rows.close()
            self.rows = None


def _util_rows(w: RunOnceWorkload, placed_node: np.ndarray, zeros=_zeros):
    """ca_util_node / ca_util_pod rows of the snapshot after FilterOutSchedulable: each
    node's running pods, then the pods placed on it (NodeInfo.Pods order).  `zeros(key, n,
    dtype)` allocates the row arrays (a caller that uploads them passes page-locked ones)."""
    f = w.filt
    n = len(f.nodes)
    nodes = zeros("nodes", n, abi.UTIL_NODE_DTYPE)
    nodes["alloc_milli"][:, 0] = f.nodes["alloc_milli_cpu"]
    nodes["alloc_milli"][:, 1] = f.nodes["alloc_memory"] * 1000
    nodes["flags"] = abi.CA_UNODE_HAS_CPU | abi.CA_UNODE_HAS_MEM
    run_pods = f.table.pods
    pend = f.pending.pods
    placed = np.nonzero(placed_node >= 0)[0]                      # positions in the filter order
    pend_ids = f.order[placed]
    all_node = np.concatenate([f.pod_node, placed_node[placed]]).astype(np.int64)
    cpu = np.concatenate([run_pods["req_milli_cpu"], pend["req_milli_cpu"][pend_ids]])
    mem = np.concatenate([run_pods["req_memory"], pend["req_memory"][pend_ids]])
    order = np.argsort(all_node, kind="stable")                   # node by node, running pods first
    pods = zeros("pods", len(order), abi.UTIL_POD_DTYPE)
    pods["req_milli"][:, 0] = cpu[order]                     # MilliValue of millicores
    pods["req_milli"][:, 1] = mem[order] * 1000
    pods["flags"] = abi.CA_UPOD_MOVABLE
    off = zeros("pod_off", n + 1, np.int32)
    np.cumsum(np.bincount(all_node, minlength=n), out=off[1:])
    # mirror pod id of every util row (running pods: 0..P-1; placed pods: their new ids)
    return nodes, off, pods, order


def _util_base(w: RunOnceWorkload):
    """ca_util_node rows and the running pods' ca_util_pod rows by node (the snapshot the
    loop starts from; cached on the workload)."""
    if getattr(w, "_ubase", None) is None:
        nodes, off, pods, _ = _util_rows(w, np.full(len(w.filt.order), -1, np.int32))
        w._ubase = (nodes, off, pods)
    return w._ubase


def _util_added(w: RunOnceWorkload, placed_node: np.ndarray, zeros=_zeros):
    """(node, ca_util_pod row) of every pod FilterOutSchedulable placed, in placement order
    (`zeros(key, n, dtype)` allocates the arrays: page-locked ones are copied in place)."""
    f = w.filt
    placed = np.nonzero(placed_node >= 0)[0]
    ids = f.order[placed]
    pods = zeros("added_pods", len(placed), abi.UTIL_POD_DTYPE)
    pods["req_milli"][:, 0] = f.pending.pods["req_milli_cpu"][ids]
    pods["req_milli"][:, 1] = f.pending.pods["req_memory"][ids] * 1000
    pods["flags"] = abi.CA_UPOD_MOVABLE
    node = zeros("added_node", len(placed), np.int32)
    node[:] = placed_node[placed]
    return node, pods


class UtilInput:
    """The utilization step's input, built before its timer: the full rows of the snapshot
    after FilterOutSchedulable (``want = "full"``: the CPU port), or the loop's starting rows
    plus the pods added since (``want = "added"``: the device table keeps the starting rows
    resident, as the mirror keeps the snapshot, and receives only the additions)."""

    def __init__(self, w: RunOnceWorkload, placed_node: np.ndarray, want: str, zeros=_zeros):
        self.want = want
        if want == "added":
            self.base = _util_base(w)
            self.added_node, self.added_pods = _util_added(w, placed_node, zeros)
        else:
            self.nodes, self.off, self.pods, _ = _util_rows(w, placed_node, zeros)


def run(backend, util_fn, w: RunOnceWorkload, timers=None, row_zeros=_zeros, expand_fn=None) -> RunOnceResult:
    """One loop on `backend` (native.Mirror or pyoracle.OracleState, freshly loaded with
    W.load_filter) with `util_fn(UtilInput, now_ns) -> UTIL_INFO rows` (its attribute `want`,
    default "full", picks the input form); `row_zeros` allocates full utilization rows;
    `expand_fn(backend, podset, samples, templates)` (e.g. DeviceExpansion) replaces the
    backend's check_templates for step 2."""
    f = w.filt
    r = RunOnceResult()
    clock = time.perf_counter

    # the pending pods, resident on the device for steps 1-3 (one upload; timed with step 1)
    t = clock()
    ps = backend.podset(f.pending) if hasattr(backend, "podset") else None
    kw = {"podset": ps} if ps is not None else {}

    # 1. FilterOutSchedulable: placed pods join the snapshot
    fo = backend.filter_out_schedulable(f.pending, f.order, f.class_owner, f.hints, 0, **kw)
    r.ms["filter"] = (clock() - t) * 1e3
    r.filter_node, r.filter_evals, r.last_index = fo.node.copy(), int(fo.evals), int(fo.last_index)
    unsched = f.order[fo.node < 0]

    # 2. expansion options: CheckPredicates of every equivalence group's sample on every template
    groups = _equivalence_groups(f.pending.pods, unsched)
    samples = np.array([g[0] for g in groups], np.int32)
    t = clock()
    if expand_fn is not None and ps is not None:
        res = expand_fn(backend, ps, samples, w.templates)
    else:
        res = backend.check_templates(f.pending, samples, w.templates, **kw)
    r.ms["expansion"] = (clock() - t) * 1e3
    # a [G][E] uint8 verdict (1 = fits, the device's verdict-only form) or ca_pred_result rows
    r.options = res.astype(np.uint8) if res.dtype == np.uint8 else (res["type"] == 0).astype(np.uint8)

    # 3. Estimate of every option, one batch
    off, idx = [0], []
    for g in range(len(w.templates)):
        for e in np.nonzero(r.options[g])[0]:
            idx.extend(groups[e])
        off.append(len(idx))
    group_off = np.array(off, np.int32)
    pod_idx = np.array(idx, np.int32)
    t = clock()
    est = backend.estimate(f.pending, group_off, pod_idx, w.templates, MAX_NODES, r.last_index, **kw)
    r.ms["estimate"] = (clock() - t) * 1e3
    r.est_results, r.est_sched = est.results.copy(), est.sched_pod.copy()
    r.last_index = int(est.last_index)                 # one PredicateChecker for the whole loop
    if ps is not None:
        ps.close()

    # 4. scale-down eligibility on the snapshot after step 1
    ui = UtilInput(w, fo.node, getattr(util_fn, "want", "full"), getattr(util_fn, "zeros", row_zeros))
    t = clock()
    r.util = util_fn(ui, w.now_ns)
    r.ms["utilization"] = (clock() - t) * 1e3
    low = np.nonzero((r.util["status"] == 0) & (r.util["utilization"] < UTIL_THRESHOLD))[0].astype(np.int32)
    r.empty = low[r.util["empty"][low] != 0]
    cand = low[r.util["empty"][low] == 0]
    r.candidates = cand

    # 5. FindNodesToRemove over the non-empty candidates (pods in NodeInfo order: running
    # pods by id, then the pods FilterOutSchedulable placed, by placement)
    P = len(f.table)
    placed = np.nonzero(fo.node >= 0)[0]
    pod_node = np.concatenate([f.pod_node, fo.node[placed]]).astype(np.int64)
    pod_id = np.concatenate([np.arange(P, dtype=np.int32), fo.pod_id[placed]])
    order = np.argsort(pod_node, kind="stable")
    node_first = np.zeros(len(f.nodes) + 1, np.int64)
    np.cumsum(np.bincount(pod_node, minlength=len(f.nodes)), out=node_first[1:])
    move_off, moves = [0], []
    for c in cand.tolist():
        ids = pod_id[order[node_first[c]:node_first[c + 1]]]
        moves.append(ids)
        move_off.append(move_off[-1] + len(ids))
    move_pods = np.concatenate(moves).astype(np.int32) if moves else np.zeros(0, np.int32)
    n_ids = int(pod_id.max()) + 1 if len(pod_id) else 0
    hints = np.full(n_ids, -1, np.int32)
    t = clock()
    sw = backend.find_nodes_to_remove(cand, np.ones(len(f.nodes), np.uint8), np.zeros(len(cand), np.int32),
                                      np.array(move_off, np.int32), move_pods, hints, r.last_index)
    r.ms["sweep"] = (clock() - t) * 1e3
    r.sweep_results, r.sweep_dest = sw.results.copy(), sw.dest.copy()
    r.sweep_hints = np.asarray(sw.hints)[move_pods].copy()
    r.last_index = int(sw.last_index)
    r.ms["total"] = sum(r.ms.values())
    r.sizes = {"pending": int(len(f.order)), "placed_by_filter": int(placed.size), "unschedulable": int(len(unsched)),
               "equivalence_groups": len(groups), "options_pairs": int(r.options.size),
               "estimate_items": int(group_off[-1]), "scale_down_candidates": int(len(low)),
               "empty": int(len(r.empty)), "sweep_candidates": int(len(cand)), "pods_to_move": int(len(move_pods)),
               "removable": int(r.sweep_results["removable"].sum())}
    return r


def compare(a: RunOnceResult, b: RunOnceResult) -> dict:
    """Per-step equality of two loops' outputs (bit-exact for everything)."""
    return {
        "filter": bool(np.array_equal(a.filter_node, b.filter_node) and a.filter_evals == b.filter_evals),
        "expansion": bool(np.array_equal(a.options, b.options)),
        "estimate": bool(np.array_equal(a.est_results, b.est_results) and np.array_equal(a.est_sched, b.est_sched)),
        "utilization": a.util.tobytes() == b.util.tobytes(),
        "sweep": bool(np.array_equal(a.sweep_results, b.sweep_results) and np.array_equal(a.sweep_dest, b.sweep_dest)
                      and np.array_equal(a.sweep_hints, b.sweep_hints)),
    }


class ShardedMirror:
    """One rank's backend of a loop run with one process per GPU: every rank
    holds a replica of the snapshot (``mirror``) and applies the loop's snapshot changes
    itself (FilterOutSchedulable, the expansion check and the utilization step run on each
    replica: they mutate or read the whole snapshot); the two batches whose units shard —
    Estimate's node groups and FindNodesToRemove's candidates — run one contiguous block
    per rank (shard.estimate_sharded / shard.sweep_sharded) and every rank receives the
    whole batch's results by all-gather, so the replicas stay identical for the next step.
    ``ex`` is the rank's shard.Exchange (RCCL or gloo all-gathers)."""

    def __init__(self, mirror, ex, rank: int, world: int):
        self.m = mirror
        self.ex = ex
        self.rank = rank
        self.world = world
        self.stats = {}

    def __getattr__(self, k):                     # podset, filter_out_schedulable, h, lib, ...
        return getattr(self.m, k)

    def estimate(self, table, group_off, pod_idx, templates, max_nodes, last_index=0, want_nodes=False, podset=None):
        from . import native, shard
        off = np.ascontiguousarray(group_off, np.int32)
        blocks = shard.split_blocks(np.diff(off), self.world)
        a, b = blocks[self.rank], blocks[self.rank + 1]
        with native.EstimatePlan(self.m, table, (off[a:b + 1] - off[a]).astype(np.int32), pod_idx[off[a]:off[b]],
                                 templates[a:b], podset=podset) as plan:
            res, sched, L, reruns = shard.estimate_sharded(plan, max_nodes, last_index, self.ex, self.rank, blocks, off)
        self.stats["estimate_reruns"] = reruns
        return native.EstimateOutput(res, sched, None, L)

    def find_nodes_to_remove(self, candidates, dest_mask, cand_status, move_off, move_pods, hints, last_index=0):
        from . import native, shard
        off = np.ascontiguousarray(move_off, np.int32)
        blocks = shard.split_blocks(np.diff(off), self.world)
        a, b = blocks[self.rank], blocks[self.rank + 1]
        h = np.array(hints, dtype=np.int32, copy=True)
        with native.RemovalPlan(self.m, candidates[a:b], dest_mask, cand_status[a:b],
                                (off[a:b + 1] - off[a]).astype(np.int32), move_pods[off[a]:off[b]]) as plan:
            sb, ph = shard.sweep_setup(plan, self.ex, self.rank, a == b)
            res, dest, L, st = shard.sweep_sharded(plan, last_index, h, len(dest_mask), self.ex, self.rank, blocks, off,
                                                   move_pods, sb, ph)
        self.stats["sweep"] = {k: v for k, v in st.items() if k in ("reached", "serial_blocks")}
        return native.RemovalOutput(res, dest, h, L)
