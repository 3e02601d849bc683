#!/usr/bin/env python3
"""bench.py — BASELINE.json's metric on its C2 configuration.

One step = one Estimate batch: BinpackingNodeEstimator.Estimate for every node
group of a scale-up (CA/core/scaleup/orchestrator/orchestrator.go:139-178), i.e. the
C2 workload of SURVEY.md §8d: 50k heterogeneous pending pods x 100 node-group
templates, resource-fit only, maxNodes = 1000 (the --max-nodes-per-scaleup
default), 1000 existing nodes, inputs resident in HBM.  The step runs the device
sort, the per-group First-Fit-Decreasing chains and the lastIndex fix-up, and returns
what Estimate returns (estimator.go:40-42) — every group's node count and scheduled
pods in placement order — on the host (§8d: Estimate latency = results on the host;
the zero-copy publisher streams them into page-locked memory while the chains run).
extra.device_resident times the same step with the scheduled pods left in HBM.

value = filter-chain evaluations the reference algorithm performs in that batch
(every RunFilterPlugins call, counted exactly) / wall time.  With --gpus N (one process
per GPU) the batch holds 100 x N node groups and each rank runs its own 100 (weak
scaling: node groups are independent units coupled only through the checker's lastIndex,
chained by one RCCL all_gather of a 4-int record per rank per step); value =
all ranks' evaluations / the slowest rank's time.  CASIM_BENCH_SCALING=strong splits the
same 100 groups over the N GPUs instead (rank 0 drives them through
ca_multi_estimate_plan_run, or CASIM_BENCH_MULTI=rccl: one block per rank).

At N > 1 the line also carries the configs that name several GPUs, every rank running one
contiguous block of units on its own mirror replica (one process per GPU, RCCL all-gathers
over xGMI): extra.c3_multi (BASELINE configs[2]: the C3 sweep's candidates, the blocks'
lastIndex chain composed in the phases of casim.h "one process per GPU"), extra.c4_multi
(configs[3]: the C4 Estimate batch's node groups) and extra.c5_runonce_multi (configs[4]:
one C5 RunOnce, Estimate and the sweep sharded), each with results_identical_to_1gpu, the
collective bytes and the CPU port's time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       (--gpus N > 1 without WORLD_SIZE starts N ranks under torch.distributed.run itself;
       with WORLD_SIZE set it must equal N.  Fewer GPUs than ranks: the ranks share devices
       and use gloo — a rehearsal, said so in config.devices)
       torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "pod×node predicate evals/sec; Estimate() latency, 50k pods × 100 node groups"
HBM_PEAK_GBS = 8000.0            # MI355X HBM3E (MI355X_MICROARCH.md, chip table)
BYTES_PER_EVAL = 64              # node record read per resource-only evaluation

# Algorithmic HBM bytes per (pod, group) item of each Estimate phase,
# bucket-sort path (score classes <= 4096):
#   score   k_class_rank: per class, not per item (0)
#   merge   k_radix_hist + k_radix_scatter, per 8-bit pass: 2 x (pod_idx 4 + class 4 + rank 4)
#           + position write 4
#   emit    k_emit_bucket: position 4 + pod_idx 4 + PodHot 32 + StreamPod write 32 + pod id 4
#           + head bit
#   chain   k_ffd_chain: StreamPod read 32 + result write 4
#   compact k_copy_segments: pod id read 4 + sched_pod write 4
PHASE_BYTES = {"score_ms": 0.0, "merge_ms": 28.0, "emit_ms": 76.125, "chain_ms": 36.0, "compact_ms": 8.0}
PHASE_KERNEL = {"score_ms": "k_class_rank", "merge_ms": "k_radix_hist+k_radix_scan+k_radix_scatter",
                "emit_ms": "k_emit_bucket", "chain_ms": "k_ffd_chain", "compact_ms": "k_copy_segments"}


def native_device_count() -> int:
    from autoscaler_amd import native
    return native.device_count()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--pods", type=int, default=50_000)
    ap.add_argument("--groups", type=int, default=100)
    ap.add_argument("--existing", type=int, default=1000)
    ap.add_argument("--max-nodes", type=int, default=1000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--with-nodes", action="store_true",
                    help="also copy each scheduled pod's new-node ordinal to the host (not part of Estimate's "
                         "Go return value (int, []*Pod), estimator.go:40-42)")
    ap.add_argument("--cpu-groups", type=int, default=100, help="groups in the bounded CPU-baseline sample")
    ap.add_argument("--no-sweep", action="store_true", help="skip the C3 scale-down sweep leg (N=1 only)")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 taint/affinity Estimate leg (N=1 only)")
    ap.add_argument("--no-expansion", action="store_true", help="skip the expansion-option feasibility leg (N=1)")
    ap.add_argument("--no-util", action="store_true", help="skip the scale-down eligibility leg (N=1)")
    ap.add_argument("--no-filter", action="store_true", help="skip the FilterOutSchedulable leg (N=1)")
    ap.add_argument("--no-unlimited", action="store_true", help="skip the C2 max_nodes=0 leg (N=1)")
    ap.add_argument("--no-runonce", action="store_true", help="skip the C5 end-to-end RunOnce leg (N=1)")
    ap.add_argument("--no-planner", action="store_true", help="skip the planner (canPersist=true) leg (N=1)")
    ap.add_argument("--sweep-nodes", type=int, default=5000)
    return ap.parse_args()


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def c4_leg(args, device: int, with_cpu: bool) -> dict:
    """C4 (BASELINE configs[3]): the Estimate batch with taints (20 classes),
    64 label pairs over 12 keys, nodeSelectors and required node-affinity terms; group pod
    lists are the pods passing CheckPredicates on the template."""
    from autoscaler_amd import native
    from autoscaler_amd import workloads as W
    w = W.c4(n_pods=args.pods, n_groups=args.groups, n_existing=args.existing, max_nodes=args.max_nodes)
    m = native.Mirror(device)
    W.load_estimate(m, w)
    out = {"workload": f"C4: {args.pods} pods x {args.groups} groups, taints/labels/affinity, "
                       f"{int(w.group_off[-1])} (pod, group) items"}
    with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
        for _ in range(2):
            plan.run(w.max_nodes, 0, copy=False, device_results=True)
        ts = []
        for _ in range(max(args.steps, 5)):
            r = None                  # (the previous result is freed outside the timing)
            t = time.perf_counter()
            r = plan.run(w.max_nodes, 0, copy=False, device_results=True)     # results in HBM, as the C2 line
            ts.append(time.perf_counter() - t)
        ms = float(np.median(ts) * 1e3)
        evals = int(r.results["evals"].sum())
        out.update({"estimate_ms": ms, "evals": evals, "evals_per_s": evals / (ms / 1e3)})
        res, sp = r.results.copy(), plan.fetch()
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle                                           # CPU baseline leg only
        o = pyoracle.OracleState()
        W.load_estimate(o, w)
        ro = None                  # (the previous result is freed outside the timing)
        t = time.perf_counter()
        ro = o.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 0)
        cpu_ms = (time.perf_counter() - t) * 1e3
        out.update({"cpu_ms": cpu_ms, "speedup": cpu_ms / ms,
                    "parity": bool(np.array_equal(ro.results, res) and np.array_equal(ro.sched_pod, sp)),
                    "cpu_baseline": {"kind": "port", "cores": 1,
                                     "sample": f"oracle/casim_oracle.c, the same C4 batch, 1 thread of {cpu_model()}"}})
    m.close()
    return out


def expansion_leg(args, device: int, with_cpu: bool) -> dict:
    """ComputeExpansionOption's feasibility for every (node group, pod group) pair
    (orchestrator.go:455-481) on the C4 attributes: CheckPredicates of
    each pod group's sample on a fresh copy of each template (ca_check_templates).
    'groups' = the distinct pod records (equivalence groups), 'all' = every pod its own
    group (no controller: the worst case)."""
    from autoscaler_amd import abi, native
    from autoscaler_amd import workloads as W
    w = W.c4(n_pods=args.pods, n_groups=args.groups, n_existing=args.existing, max_nodes=args.max_nodes)
    pods = w.table.pods
    uniq = np.unique(pods.view(np.dtype((np.void, pods.dtype.itemsize))), return_index=True)[1].astype(np.int32)
    m = native.Mirror(device)
    W.load_estimate(m, w)
    out = {"workload": f"C4 pods x {args.groups} node-group templates"}
    podset = native.PodSet(m, w.table)                                      # pods resident in HBM
    for name, samples in (("groups", np.sort(uniq)), ("all", np.arange(len(pods), dtype=np.int32))):
        # the verdicts (which pod groups join which option) into page-locked memory, then
        # the full results (failing plugin and reasons per pair: eg.SchedulingErrors)
        pin = native.PinnedArray(m.lib, len(samples) * len(w.templates), np.uint8)
        ok = pin.array.reshape(len(w.templates), len(samples))
        pin_full = native.PinnedArray(m.lib, len(samples) * len(w.templates), abi.PRED_RESULT_DTYPE)
        full = pin_full.array.reshape(len(w.templates), len(samples))
        rec = {"pod_groups": int(len(samples)), "pairs": int(len(samples) * len(w.templates))}
        for mode in ("verdicts", "with_reasons"):
            call = (lambda: m.check_templates(w.table, samples, w.templates, podset=podset, verdict_only=True,
                                              out=ok)) if mode == "verdicts" else \
                   (lambda: m.check_templates(w.table, samples, w.templates, podset=podset, out=full))
            call()                                                         # warm-up
            ts = []
            for _ in range(max(args.steps, 5)):
                res = None                  # (the previous result is freed outside the timing)
                t = time.perf_counter()
                res = call()
                ts.append(time.perf_counter() - t)
            ms = float(np.median(ts) * 1e3)
            rec[f"{mode}_ms"] = ms
            rec[f"{mode}_pairs_per_s"] = len(samples) * len(w.templates) / (ms / 1e3)
        # the same with the node groups resident (ca_expansion_plan): the samples in and the
        # results out through page-locked memory the kernel reads and writes in place
        res = res.copy()                                                   # (the resident runs reuse `full`)
        with native.ExpansionPlan(m, w.templates) as plan:
            for mode in ("verdicts", "with_reasons"):
                call = (lambda: plan.run(podset, samples, verdict_only=True, out=ok)) if mode == "verdicts" else \
                       (lambda: plan.run(podset, samples, out=full))
                call()
                ts, ks = [], []
                for _ in range(max(args.steps, 5)):
                    r2 = None                  # (the previous result is freed outside the timing)
                    t = time.perf_counter()
                    r2 = call()
                    ts.append(time.perf_counter() - t)
                    ks.append(plan.kernel_ms)
                rec[f"resident_{mode}_ms"] = float(np.median(ts) * 1e3)
                rec[f"resident_{mode}_kernel_ms"] = float(np.median(ks))
            rec["resident_matches"] = bool(np.array_equal(r2, res))
        rec["feasible_pairs"] = int((res["type"] == 0).sum())
        rec["verdicts_match_results"] = bool(np.array_equal(ok.astype(bool), res["type"] == 0))
        res = res.copy()
        pin.close()
        pin_full.close()
        ms = rec["verdicts_ms"]
        if with_cpu:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle                                           # CPU baseline leg only
            o = pyoracle.OracleState()
            W.load_estimate(o, w)
            ro = None                  # (the previous result is freed outside the timing)
            t = time.perf_counter()
            ro = o.check_templates(w.table, samples, w.templates)
            cpu_ms = (time.perf_counter() - t) * 1e3
            rec.update({"cpu_ms": cpu_ms, "speedup_verdicts": cpu_ms / ms,
                        "speedup_with_reasons": cpu_ms / rec["with_reasons_ms"],
                        "speedup_resident_verdicts": cpu_ms / rec["resident_verdicts_ms"],
                        "speedup_resident_with_reasons": cpu_ms / rec["resident_with_reasons_ms"],
                        "parity": bool(np.array_equal(ro, res))})
        out[name] = rec
    podset.close()
    out["includes"] = ("host->device template rows, the matrix kernel, device->host results (1 B per pair, or 16 B "
                       "per pair with reasons, into page-locked memory)")
    if with_cpu:
        out["cpu_baseline"] = {"kind": "port", "cores": 1,
                               "sample": f"oracle/casim_oracle.c or_check_templates (fork, template copy, "
                                         f"CheckPredicates, revert per node group), 1 thread of {cpu_model()}"}
    m.close()
    return out


def utilization_leg(args, device: int, with_cpu: bool) -> dict:
    """Scale-down eligibility at C5 size: utilization.Calculate
    (info.go:48-127) + the FindEmptyNodesToRemove verdict for 15k nodes / ~300k pods in one
    launch (ca_util_calculate), table resident in HBM, results left in HBM.  Roofline: HBM,
    algorithmic bytes = node row 32 B + offset 4 B + result 48 B per node, 48 B per pod."""
    from autoscaler_amd import native
    from autoscaler_amd import workloads as W
    nodes, off, pods, now = W.util_table(seed=11, n_nodes=15000, pods_per_node=20)
    t = native.UtilTable(device, nodes, off, pods)
    for _ in range(3):
        t.calculate(True, True, now, to_host=False)
    kms, wall = [], []
    for _ in range(max(args.steps, 20)):
        t0 = time.perf_counter()
        t.calculate(True, True, now, to_host=False)
        wall.append(time.perf_counter() - t0)
        kms.append(t.kernel_ms)
    got = t.calculate(True, True, now)
    t.close()
    k = float(np.mean(kms))
    algo = 84 * len(nodes) + 4 + 48 * len(pods)
    out = {"workload": f"C5 nodes: {len(nodes)} nodes, {len(pods)} pods (ragged 0-40 per node), skip DaemonSet "
                       f"and mirror pods", "kernel": "k_node_utilization", "kernel_ms": k,
           "call_ms": float(np.median(wall) * 1e3), "nodes_per_s": len(nodes) / (k / 1e3),
           "roofline": {"bound": "hbm", "achieved": algo / (k / 1e3) / 1e9, "peak": 8000.0, "unit": "GB/s",
                        "frac": algo / (k / 1e3) / 1e9 / 8000.0, "bytes_per_launch": algo, "traffic": None}}
    tf = os.path.join(ROOT, "profiles", "pmc_util_traffic.json")     # rocprofv3 --pmc passes (scripts/pmc_util.py)
    if os.path.exists(tf):
        with open(tf) as f:
            kt = json.load(f)["kernels"].get("k_node_utilization")
        if kt:
            out["roofline"]["traffic"] = kt["traffic_bytes_per_launch"]
            out["roofline"]["traffic_source"] = "profiles/pmc_util_traffic.json (FETCH_SIZE x2 + WRITE_SIZE, per launch)"
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle                                           # CPU baseline leg only
        t0 = time.perf_counter()
        ref = pyoracle.node_utilization(nodes, off, pods, True, True, now)
        cpu_ms = (time.perf_counter() - t0) * 1e3
        out.update({"cpu_ms": cpu_ms, "speedup_kernel": cpu_ms / k, "parity": got.tobytes() == ref.tobytes(),
                    "cpu_baseline": {"kind": "port", "cores": 1,
                                     "sample": f"oracle/casim_oracle.c or_node_utilization, the same table, 1 thread "
                                               f"of {cpu_model()}"}})
    return out


def filter_leg(args, device: int, with_cpu: bool) -> dict:
    """FilterOutSchedulable (filter_out_schedulable.go:95-124) on C5: 15k nodes
    running 300k pods, 20k pending pods in priority order, TrySchedulePods(ScheduleAnywhere,
    breakOnFailure=false) with hints and the similar-pods cache, one ca_filter_out_schedulable
    call per step inside a fork that is reverted after it (mirror resident in HBM).
    'c5-c4' adds the C4 taint/label universe; 'loose' is the same cluster at 20-70 %
    utilisation (nearly every pod fits its first node: the port does ~1 evaluation per pod,
    the regime where the one-wavefront walk does not beat it)."""
    from autoscaler_amd import native
    from autoscaler_amd import workloads as W
    out = {}
    for name, kw in (("c5", {}), ("c5-c4", {"taints": True}), ("loose", {"util_low": (0.2, 0.4), "util_high": (0.5, 0.7)})):
        w = W.c5_filter(**kw)
        g = native.Mirror(device)
        W.load_filter(g, w)
        ts, ks = [], []
        for rep in range(1 + max(3, min(args.steps, 5))):
            g.fork()
            rg = None                  # (the previous result is freed outside the timing)
            t = time.perf_counter()
            rg = g.filter_out_schedulable(w.pending, w.order, w.class_owner, w.hints, 0)
            dt = (time.perf_counter() - t) * 1e3
            st = g.filter_stats()
            g.revert()
            if rep:                                               # first call is the warm-up
                ts.append(dt)
                ks.append(st["kernel_ms"])
        ms = float(np.median(ts))
        rec = {"workload": f"{name}: {len(w.order)} pending pods over {len(w.nodes)} nodes running "
                           f"{len(w.pod_node)} pods", "call_ms": ms, "kernel_ms": float(np.median(ks)), "placed": int(rg.placed),
               "evals": int(rg.evals), "evals_per_s": rg.evals / (ms / 1e3)}
        g.close()
        if with_cpu:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle                                       # CPU baseline leg only
            o = pyoracle.OracleState()
            W.load_filter(o, w)
            o.fork()
            ro = None                  # (the previous result is freed outside the timing)
            t = time.perf_counter()
            ro = o.filter_out_schedulable(w.pending, w.order, w.class_owner, w.hints, 0)
            cpu_ms = (time.perf_counter() - t) * 1e3
            rec.update({"cpu_ms": cpu_ms, "speedup": cpu_ms / ms,
                        "parity": bool(np.array_equal(rg.node, ro.node) and rg.evals == ro.evals
                                       and rg.last_index == ro.last_index and np.array_equal(rg.hints, ro.hints))})
        out[name] = rec
    if with_cpu:
        out["cpu_baseline"] = {"kind": "port", "cores": 1,
                               "sample": f"oracle/casim_oracle.c or_filter_out_schedulable, the same call, 1 thread "
                                         f"of {cpu_model()}"}
    return out


def sweep_leg(args, device: int, with_cpu: bool) -> dict:
    """C3 (BASELINE configs[2]): FindNodesToRemove over a 5k-node cluster with
    150k running pods, legacy semantics, inputs resident in HBM (ca_removal_plan) and the
    HintingSimulator's hints resident in the mirror.  'fresh' = first loop (no hints),
    'hinted' = a following loop (the previous loop's hints: the steady state)."""
    from autoscaler_amd import native
    from autoscaler_amd import workloads as W
    w = W.c3(n_nodes=args.sweep_nodes)
    m = native.Mirror(device)
    W.load_sweep(m, w)
    sweep_args = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
    fresh_h = np.full(len(w.table), -1, np.int32)
    out = {"workload": f"C3: {args.sweep_nodes} nodes, {len(w.table)} running pods, candidates = all nodes",
           "inputs": "resident in HBM (removal plan); hints resident in the mirror"}
    with native.RemovalPlan(m, *sweep_args) as plan:
        runs = {}
        for mode in ("fresh", "hinted"):
            ts = []
            # untimed warm-up: the first call of a shape runs eagerly, the second captures the
            # HIP graph, the first replay sets it up; the timed calls are the steady state
            for it in range(max(args.warmup, 3) + max(args.steps, 10)):
                if mode == "fresh":
                    m.set_hints(fresh_h)
                r = None                  # (the previous result is freed outside the timing)
                t = time.perf_counter()
                r = plan.run(0)
                if it >= max(args.warmup, 3):
                    ts.append(time.perf_counter() - t)
            runs[mode] = (r, m.get_hints(len(w.table)))
            out[f"{mode}_ms"] = float(np.median(ts) * 1e3)
            out[f"{mode}_evals"] = int(r.results["evals"].sum())
            out[f"{mode}_removable"] = int(r.results["removable"].sum())
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle                                           # CPU baseline leg only
        o = pyoracle.OracleState()
        W.load_sweep(o, w)
        h = fresh_h
        for mode in ("fresh", "hinted"):
            cts = []
            for _ in range(3):                                    # median, as on the GPU side
                ro = None                  # (the previous result is freed outside the timing)
                t = time.perf_counter()
                ro = o.find_nodes_to_remove(*sweep_args, h, 0)
                cts.append(time.perf_counter() - t)
            cpu_ms = float(np.median(cts) * 1e3)
            r, hg = runs[mode]
            out[f"{mode}_cpu_ms"] = cpu_ms
            out[f"{mode}_speedup"] = cpu_ms / out[f"{mode}_ms"]
            out[f"{mode}_parity"] = bool(np.array_equal(ro.results, r.results) and ro.last_index == r.last_index
                                         and np.array_equal(ro.hints, hg))
            h = ro.hints
        out["cpu_baseline"] = {"kind": "port", "cores": 1,
                               "sample": f"oracle/casim_oracle.c FindNodesToRemove, same C3 sweep, 1 thread of "
                                         f"{cpu_model()}"}
    m.close()
    return out


def planner_leg(args, device: int, with_cpu: bool) -> dict:
    """The planner's committing loop (canPersist=true, planner.go:252-296) on C3 through
    ca_plan_removals, inside a fork reverted after each run (UpdateClusterState does the
    same), at three unneeded-node limits: 20 (the first loop's limit with the default
    MaxScaleDownParallelism 10, planner.go:318-334), 200, and none."""
    from autoscaler_amd import native
    from autoscaler_amd import workloads as W
    w = W.c3(n_nodes=args.sweep_nodes)
    args_ = (w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods)
    hints = np.full(len(w.table), -1, np.int32)
    out = {"workload": f"C3: {args.sweep_nodes} nodes, {len(w.table)} running pods, candidates = all nodes in order",
           "runs": {}}
    firsts = {}
    for limit in (20, 200, 0):
        m = native.Mirror(device)                   # fresh: the copies' ids then match the port's
        W.load_sweep(m, w)
        ts, st, split = [], None, []
        for _ in range(9):                          # the first run also uploads the snapshot; the median of
                                                    # eight warm runs (a host stall of 10-40 ms hits one or two)
            m.fork()
            r = None                  # (the previous result is freed outside the timing)
            t = time.perf_counter()
            r = m.plan_removals(*args_, hints, 0, limit)
            ts.append(time.perf_counter() - t)
            st = m.plan_stats()
            if st["path"] == "chain":
                split.append(m.plan_chain_profile())
            m.revert()
            firsts.setdefault(limit, r)
        out["runs"][str(limit)] = {"gpu_ms": float(np.median(ts[1:]) * 1e3), "min_ms": float(np.min(ts[1:]) * 1e3),
                                   "path": st["path"], "rounds": st["rounds"],
                                   "conflicts": st["conflicts"], "simulated": st["simulated"],
                                   "removable": int(r.results["removable"].sum()),
                                   "candidates_run": int((r.results["reason"] != 101).sum()),
                                   "all_ms": [round(x * 1e3, 3) for x in ts]}
        if split:                                   # library-side split of the call (median over the warm runs)
            out["runs"][str(limit)]["split_ms"] = {
                k: float(np.median([s[k] for s in split[1:] or split]))
                for k in ("sync_ms", "launch_kernel_ms", "kernel_ms", "readback_ms", "replay_ms")}
        m.close()
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle                                           # CPU baseline leg only
        for limit in (20, 200, 0):
            o = pyoracle.OracleState()
            W.load_sweep(o, w)
            cts, ro = [], None
            for _ in range(3):                                    # median, as on the GPU side
                o.fork()
                r1 = None                  # (the previous result is freed outside the timing)
                t = time.perf_counter()
                r1 = o.plan_removals(*args_, hints, 0, limit)
                cts.append(time.perf_counter() - t)
                o.revert()
                ro = ro or r1
            run = out["runs"][str(limit)]
            run["cpu_ms"] = float(np.median(cts) * 1e3)
            run["speedup"] = run["cpu_ms"] / run["gpu_ms"]
            g = firsts[limit]
            run["parity"] = bool(np.array_equal(ro.results, g.results) and np.array_equal(ro.moves, g.moves)
                                 and np.array_equal(ro.hints, g.hints) and ro.last_index == g.last_index)
        out["cpu_baseline"] = {"kind": "port", "cores": 1,
                               "sample": f"oracle/casim_oracle.c or_plan_removals, same loop, median of 3 runs (inside a "
                                         f"reverted fork; the GPU's is the median of 8 warm runs), 1 thread of {cpu_model()}"}
    return out


def runonce_leg(args, device: int, with_cpu: bool) -> dict:
    """C5 end to end (autoscaler_amd/runonce.py): one RunOnce's simulation legs over 15k
    nodes / 300k pods / 20k pending pods — FilterOutSchedulable, expansion options (100 node
    groups), Estimate of every option, utilization + empty nodes, FindNodesToRemove over the
    low-utilization candidates — each step through the C ABI, inside a fork reverted after
    the loop; the CPU port runs the same loop."""
    from autoscaler_amd import native, runonce
    from autoscaler_amd import workloads as W
    w = runonce.c5_runonce()
    m = native.Mirror(device)
    W.load_filter(m, w.filt)

    # the utilization table holds the loop's starting snapshot resident (as the mirror does)
    # and receives the pods FilterOutSchedulable added (ca_util_table_set_added)
    util = runonce.DeviceUtil(device)
    # the node groups' templates stay resident across loops (ca_expansion_plan)
    expand = runonce.DeviceExpansion()
    runs = []
    for _ in range(1 + max(2, min(args.steps, 4))):
        m.fork()
        runs.append(runonce.run(m, util, w, expand_fn=expand))
        m.revert()
    expand.close()
    util.close()
    m.close()
    keys = list(runs[-1].ms)
    out = {"workload": "C5 RunOnce: 15000 nodes, 300000 running pods, 20000 pending (15% of the controller "
                       "variants too large for existing nodes), 100 node groups",
           "sizes": runs[-1].sizes,
           "gpu_ms": {k: float(np.median([r.ms[k] for r in runs[1:]])) for k in keys}}
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle                                           # CPU baseline leg only
        o = pyoracle.OracleState()
        W.load_filter(o, w.filt)
        ro = runonce.run(o, pyoracle.runonce_cpu_util, w)
        out["cpu_ms"] = ro.ms
        out["speedup"] = {k: ro.ms[k] / out["gpu_ms"][k] for k in keys if out["gpu_ms"][k] > 0}
        out["parity"] = runonce.compare(ro, runs[-1])
        out["cpu_baseline"] = {"kind": "port", "cores": 1,
                               "sample": f"oracle/casim_oracle.c, the same loop step by step, 1 thread of {cpu_model()}"}
    return out


class RankCtx:
    """One rank of a --gpus N > 1 run: torch.distributed handle, rank, world, device,
    collective device and the byte all-gather (RCCL over xGMI; gloo when ranks share a
    device in a rehearsal)."""

    def __init__(self, dist, rank, world, local, coll_dev, shared):
        from autoscaler_amd import shard
        self.dist, self.rank, self.world, self.local, self.coll_dev = dist, rank, world, local, coll_dev
        self.shared = shared
        self.gather = shard.torch_gather_bytes(dist, coll_dev)

    def timed(self, fn, steps: int, warmup: int):
        """fn() `warmup` times, then `steps` times between barrier + device syncs; returns
        (max over ranks of the elapsed seconds, last output)."""
        import torch
        out = None
        for _ in range(warmup):
            out = fn()
        self.dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = fn()
        torch.cuda.synchronize()
        self.dist.barrier()
        el = time.perf_counter() - t0
        t = torch.tensor([el], dtype=torch.float64, device=self.coll_dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t[0]), out


def _devices_note(ctx) -> str:
    return (f"{ctx.world} ranks sharing {native_device_count()} device(s) (rehearsal, gloo collectives)"
            if ctx.shared else f"{ctx.world} ranks, one GPU each, RCCL all-gathers over xGMI")


def c3_multi_leg(args, ctx) -> dict:
    """BASELINE configs[2] at N > 1: the C3 FindNodesToRemove sweep (5k nodes, 150k pods)
    with its candidates in N contiguous blocks, one per rank (cluster.go:130-137),
    each rank on its own mirror replica; the blocks' lastIndex chain composed in three
    phases (casim.h "one process per GPU": PROBE, MAP, ca_sweep_compose, RESOLVE) and one
    all-gather of every block's results, destinations and hints (shard.sweep_sharded).
    One step = one whole sweep, results and hints on every rank.  'fresh' = the first loop,
    'hinted' = the next loop from the first loop's hints."""
    from autoscaler_amd import native, shard
    from autoscaler_amd import workloads as W
    w = W.c3(n_nodes=args.sweep_nodes)
    R, rank = ctx.world, ctx.rank
    blocks = shard.split_blocks(np.diff(w.move_off), R)
    a, b = blocks[rank], blocks[rank + 1]
    m = native.Mirror(ctx.local)
    W.load_sweep(m, w)
    plan = native.RemovalPlan(m, w.candidates[a:b], w.dest_mask, w.cand_status[a:b],
                              (w.move_off[a:b + 1] - w.move_off[a]).astype(np.int32),
                              w.move_pods[w.move_off[a]:w.move_off[b]])
    ex = shard.Exchange(ctx.gather)
    sb, ph = shard.sweep_setup(plan, ex, rank, a == b)
    n = len(w.nodes)
    fresh = np.full(len(w.table), -1, np.int32)
    steps = max(args.steps, 10)
    out = {"workload": f"C3: {args.sweep_nodes} nodes, {len(w.table)} running pods, candidates = all nodes, "
                       f"in {R} contiguous blocks (candidates {blocks})",
           "devices": _devices_note(ctx), "scaling": "strong (the same sweep over N GPUs)"}
    h_in, L_in = fresh, 0
    runs = {}
    for mode in ("fresh", "hinted"):
        hh = {}

        def step():
            h = h_in.copy()
            r = shard.sweep_sharded(plan, L_in, h, n, ex, rank, blocks, w.move_off, w.move_pods, sb, ph)
            hh["h"] = h
            return r
        b0, c0 = ex.bytes, ex.calls
        el, (res, dest, L, st) = ctx.timed(step, steps, max(args.warmup, 3))
        per = steps + max(args.warmup, 3)
        runs[mode] = (res, dest, L, hh["h"], h_in, L_in)
        out[f"{mode}_ms"] = el / steps * 1e3
        out[f"{mode}_blocks_composed"] = st["reached"]
        out[f"{mode}_blocks_serial"] = st["serial_blocks"]
        out[f"{mode}_collective_bytes_per_rank"] = (ex.bytes - b0) / per
        out[f"{mode}_collectives"] = (ex.calls - c0) / per
        out[f"{mode}_removable"] = int(res["removable"].sum())
        h_in, L_in = hh["h"], L
    plan.close()
    if rank == 0:
        # the same sweeps on one GPU (one plan over every candidate, this rank's mirror)
        with native.RemovalPlan(m, w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods) as one:
            same = True
            for mode in ("fresh", "hinted"):
                res, dest, L, h_out, h0, L0 = runs[mode]
                ts = []
                for _ in range(5):
                    h = h0.copy()
                    t0 = time.perf_counter()
                    r1 = one.run(L0, hints=h, want_dest=True)
                    ts.append(time.perf_counter() - t0)
                out[f"{mode}_1gpu_ms"] = float(np.median(ts) * 1e3)
                same &= bool(np.array_equal(r1.results, res) and np.array_equal(r1.dest, dest)
                             and r1.last_index == L and np.array_equal(h, h_out))
            out["results_identical_to_1gpu"] = same
        if not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle                                           # CPU baseline leg only
            o = pyoracle.OracleState()
            W.load_sweep(o, w)
            par = True
            for mode in ("fresh", "hinted"):
                res, dest, L, h_out, h0, L0 = runs[mode]
                t0 = time.perf_counter()
                ro = o.find_nodes_to_remove(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods, h0, L0)
                out[f"{mode}_cpu_ms"] = (time.perf_counter() - t0) * 1e3
                out[f"{mode}_speedup"] = out[f"{mode}_cpu_ms"] / out[f"{mode}_ms"]
                par &= bool(np.array_equal(ro.results, res) and np.array_equal(ro.dest, dest) and ro.last_index == L
                            and np.array_equal(ro.hints, h_out))
            out["parity_vs_oracle"] = par
            out["cpu_baseline"] = {"kind": "port", "cores": 1,
                                   "sample": f"oracle/casim_oracle.c FindNodesToRemove, the same C3 sweeps, 1 thread of "
                                             f"{cpu_model()}"}
    m.close()
    return out


def c4_multi_leg(args, ctx) -> dict:
    """BASELINE configs[3] at N > 1: the C4 Estimate batch (50k pods x 100 groups, taints,
    labels, node affinity) with its node groups in N contiguous blocks balanced by items,
    one per rank on its own mirror replica, the lastIndex chain by all-gathers of a 4-int
    record (a sensitive block run from a wrong input runs again; others are re-based), then
    two all-gathers bring every rank the per-group records and scheduled pods
    (shard.estimate_sharded).  One step = the whole batch, results on every rank's host."""
    from autoscaler_amd import native, shard
    from autoscaler_amd import workloads as W
    w = W.c4(n_pods=args.pods, n_groups=args.groups, n_existing=args.existing, max_nodes=args.max_nodes)
    R, rank = ctx.world, ctx.rank
    blocks = shard.split_blocks(np.diff(w.group_off), R)
    a, b = blocks[rank], blocks[rank + 1]
    off = w.group_off
    m = native.Mirror(ctx.local)
    W.load_estimate(m, w)
    plan = native.EstimatePlan(m, w.table, (off[a:b + 1] - off[a]).astype(np.int32), w.pod_idx[off[a]:off[b]],
                               w.templates[a:b])
    ex = shard.Exchange(ctx.gather)
    steps = max(args.steps, 5)
    b0, c0 = ex.bytes, ex.calls
    rr = {"n": 0}

    def step():
        r = shard.estimate_sharded(plan, w.max_nodes, 0, ex, rank, blocks, off)
        rr["n"] += r[3]
        return r
    el, (res, sched, L, _) = ctx.timed(step, steps, 2)
    per = steps + 2
    items = int(off[-1])
    evals = int(res["evals"].sum())
    out = {"workload": f"C4: {args.pods} pods x {args.groups} groups, taints/labels/affinity, {items} (pod, group) "
                       f"items, in {R} contiguous blocks (groups {blocks})",
           "devices": _devices_note(ctx), "scaling": "strong (the same batch over N GPUs)",
           "estimate_ms": el / steps * 1e3, "evals": evals, "evals_per_s": evals / (el / steps),
           "reruns_rank0": rr["n"] / per,
           "collective_bytes_per_rank": (ex.bytes - b0) / per, "collectives": (ex.calls - c0) / per}
    reruns = ex.gather(np.array([rr["n"]], np.int64))
    out["block_reruns_all_ranks"] = int(sum(int(v[0]) for v in reruns)) / per
    plan.close()
    if rank == 0:
        with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as one:
            ts = []
            for _ in range(5):
                t0 = time.perf_counter()
                o1 = one.run(w.max_nodes, 0, want_nodes=False)
                ts.append(time.perf_counter() - t0)
            out["estimate_1gpu_ms"] = float(np.median(ts) * 1e3)
            out["results_identical_to_1gpu"] = bool(np.array_equal(o1.results, res) and o1.last_index == L and all(
                np.array_equal(o1.sched_pod[off[g]:off[g] + int(o1.results[g]["n_scheduled"])],
                               sched[off[g]:off[g] + int(o1.results[g]["n_scheduled"])]) for g in range(len(off) - 1)))
        if not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle                                           # CPU baseline leg only
            o = pyoracle.OracleState()
            W.load_estimate(o, w)
            t0 = time.perf_counter()
            ro = o.estimate(w.table, w.group_off, w.pod_idx, w.templates, w.max_nodes, 0)
            out["cpu_ms"] = (time.perf_counter() - t0) * 1e3
            out["speedup"] = out["cpu_ms"] / out["estimate_ms"]
            out["parity_vs_oracle"] = bool(np.array_equal(ro.results, res) and ro.last_index == L and all(
                np.array_equal(ro.sched_pod[off[g]:off[g] + int(ro.results[g]["n_scheduled"])],
                               sched[off[g]:off[g] + int(ro.results[g]["n_scheduled"])]) for g in range(len(off) - 1)))
            out["cpu_baseline"] = {"kind": "port", "cores": 1,
                                   "sample": f"oracle/casim_oracle.c, the same C4 batch, 1 thread of {cpu_model()}"}
    m.close()
    return out


def c5_multi_leg(args, ctx) -> dict:
    """BASELINE configs[4] at N > 1: one C5 RunOnce (15k nodes, 300k pods, 20k pending,
    100 node groups) with one process per GPU (runonce.ShardedMirror): every rank applies
    FilterOutSchedulable, the expansion check and the utilization step to its replica; the
    Estimate of every option and FindNodesToRemove run one block of node groups /
    candidates per rank, results all-gathered to every rank.  One step = one loop inside a
    fork reverted after it."""
    from autoscaler_amd import native, runonce, shard
    from autoscaler_amd import workloads as W
    w = runonce.c5_runonce()
    m = native.Mirror(ctx.local)
    W.load_filter(m, w.filt)
    ex = shard.Exchange(ctx.gather)
    sm = runonce.ShardedMirror(m, ex, ctx.rank, ctx.world)
    util = runonce.DeviceUtil(ctx.local)
    expand = runonce.DeviceExpansion()
    loops = []

    def step():
        m.fork()
        r = runonce.run(sm, util, w, expand_fn=expand)
        m.revert()
        loops.append(r)
        return r
    steps = max(2, min(args.steps, 4))
    b0 = ex.bytes
    el, r = ctx.timed(step, steps, 1)
    keys = list(r.ms)
    out = {"workload": "C5 RunOnce: 15000 nodes, 300000 running pods, 20000 pending, 100 node groups; Estimate and "
                       f"FindNodesToRemove in {ctx.world} blocks (one per rank), the other legs on every replica",
           "devices": _devices_note(ctx), "scaling": "strong (the same loop over N GPUs)",
           "loop_ms": el / steps * 1e3,
           "gpu_ms_rank0": {k: float(np.median([x.ms[k] for x in loops[1:]])) for k in keys},
           "sizes": r.sizes, "sweep_blocks": sm.stats.get("sweep"),
           "collective_bytes_per_rank_per_loop": (ex.bytes - b0) / (steps + 1)}
    if ctx.rank == 0:
        m.fork()
        r1 = runonce.run(m, util, w, expand_fn=expand)           # the same loop on one GPU
        m.revert()
        out["gpu_ms_1gpu"] = r1.ms
        out["results_identical_to_1gpu"] = runonce.compare(r1, r)
        if not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle                                           # CPU baseline leg only
            o = pyoracle.OracleState()
            W.load_filter(o, w.filt)
            ro = runonce.run(o, pyoracle.runonce_cpu_util, w)
            out["cpu_ms"] = ro.ms
            out["speedup_total"] = ro.ms["total"] / out["loop_ms"]
            out["parity_vs_oracle"] = runonce.compare(ro, r)
            out["cpu_baseline"] = {"kind": "port", "cores": 1,
                                   "sample": f"oracle/casim_oracle.c, the same loop step by step, 1 thread of {cpu_model()}"}
    expand.close()
    util.close()
    m.close()
    return out


def split_groups(group_off, world: int) -> list:
    """Contiguous blocks of node groups, one per rank, balanced by (pod, group) items (the
    same split as ca_multi_estimate_plan, multi.hip:split_blocks)."""
    G = len(group_off) - 1
    w = np.maximum(np.diff(group_off), 1).astype(np.int64)
    tot, acc, b = int(w.sum()), 0, [0]
    D = max(1, min(world, G))
    for i in range(G):
        acc += int(w[i])
        k = len(b)
        if k < D and i + 1 < G and G - (i + 1) >= D - k and acc * D >= tot * k:
            b.append(i + 1)
    b.append(G)
    while len(b) < world + 1:                 # more ranks than groups: empty blocks at the end
        b.append(G)
    return b


def c2_unlimited_leg(args, device: int, with_cpu: bool) -> dict:
    """C2 with an unlimited limiter (maxNodes = 0, threshold_based_limiter.go:49-52; the
    BASELINE C2 row's second setting): new-node rows in per-group HBM slabs
    (k_ffd_chain<GROWS>), results to the host.  Parity against the committed oracle result
    (tests/golden/c2_unlimited.json: per-group fields and a CRC-32 of each scheduled list)."""
    import zlib
    from autoscaler_amd import native
    from autoscaler_amd import workloads as W
    w = W.c2()
    m = native.Mirror(device)
    W.load_estimate(m, w)
    out = {"workload": "C2 (50k pods x 100 groups, 1000 existing nodes), max_nodes = 0 (unlimited)"}
    with native.EstimatePlan(m, w.table, w.group_off, w.pod_idx, w.templates) as plan:
        plan.run(0, 0, want_nodes=False, copy=False)
        ts = []
        for _ in range(max(3, min(args.steps, 5))):
            r = None                  # (the previous result is freed outside the timing)
            t = time.perf_counter()
            r = plan.run(0, 0, want_nodes=False, copy=False)
            ts.append(time.perf_counter() - t)
        ms = float(np.median(ts) * 1e3)
        evals = int(r.results["evals"].sum())
        out.update({"ms_per_step": ms, "evals": evals, "evals_per_s": evals / (ms / 1e3),
                    "chain_kernel_ms": plan.stats()["phases"]["chain_ms"]})
        gf = os.path.join(ROOT, "tests", "golden", "c2_unlimited.json")
        if os.path.exists(gf):
            with open(gf) as f:
                gold = json.load(f)
            ok = gold["last_index"] == r.last_index
            for g, rec in enumerate(gold["groups"]):
                res = r.results[g]
                ok &= all(int(res[k]) == rec[k] for k in ("node_count", "n_scheduled", "nodes_added", "last_index_in",
                                                          "last_index_out", "status", "evals"))
                a, n = int(w.group_off[g]), int(res["n_scheduled"])
                ok &= zlib.crc32(np.ascontiguousarray(r.sched_pod[a:a + n], np.int32).tobytes()) == rec["sched_crc32"]
            out["parity_vs_golden"] = bool(ok)
    if with_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle                                           # CPU baseline leg only
        o = pyoracle.OracleState()
        W.load_estimate(o, w)
        g = 3                                                     # bounded sample: the first groups
        off = w.group_off[: g + 1]
        ro = None                  # (the previous result is freed outside the timing)
        t = time.perf_counter()
        ro = o.estimate(w.table, off, w.pod_idx[: off[-1]], w.templates[:g], 0, 0)
        cpu_s = time.perf_counter() - t
        cev = int(ro.results["evals"].sum())
        out["cpu_baseline"] = {"value": cev / cpu_s, "unit": "evals/s", "cores": 1, "kind": "port",
                               "sample": f"oracle/casim_oracle.c Estimate of the first {g} unlimited C2 groups "
                                         f"({cev} evals in {cpu_s:.2f} s), 1 thread of {cpu_model()}"}
        out["speedup_evals_per_s"] = out["evals_per_s"] / (cev / cpu_s)
    m.close()
    return out


def multi_main(args, world: int, rank: int, dist, coll_dev: str):
    """--gpus N > 1 (default): rank 0 drives all N GPUs through the C ABI's multi-device entry
    (ca_multi_estimate_plan_*: replicated mirrors, the node groups in N contiguous blocks run
    concurrently from one host thread per device, the lastIndex chain fixed up in the
    library — the path a cgo caller uses, results assembled in one process); the other ranks
    only join the barriers around the timed region.  CASIM_BENCH_MULTI=rccl: every rank
    runs its block and the chain goes over an RCCL all_gather (main below)."""
    import torch
    from autoscaler_amd import native
    from autoscaler_amd import workloads as W
    result = None
    w = W.c2(n_pods=args.pods, n_groups=args.groups, n_existing=args.existing, max_nodes=args.max_nodes, seed=42)
    items = int(w.group_off[-1])
    if rank == 0:
        ndev = max(1, native.device_count())
        mirrors = [native.Mirror(d % ndev) for d in range(world)]
        for m in mirrors:
            W.load_estimate(m, w)
        multi = native.Multi(mirrors)
        plan = native.MultiEstimatePlan(multi, w.table, w.group_off, w.pod_idx, w.templates)
        for _ in range(args.warmup):
            plan.run(w.max_nodes, 0, want_nodes=False, copy=False)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evals, out = 0, None
    if rank == 0:
        for _ in range(args.steps):
            out = plan.run(w.max_nodes, 0, want_nodes=False, copy=False)
            evals += int(out.results["evals"].sum())
    torch.cuda.synchronize()
    dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64, device=coll_dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t[0])
    if rank == 0:
        st = plan.stats()
        pods = out.sched_pod.copy()
        res = out.results.copy()
        # the same batch on one device: identical outputs (the multi path's parity)
        with native.EstimatePlan(mirrors[0], w.table, w.group_off, w.pod_idx, w.templates) as one:
            o1 = one.run(w.max_nodes, 0, want_nodes=False)
        same = bool(np.array_equal(o1.results, res) and np.array_equal(o1.sched_pod, pods)
                    and o1.last_index == out.last_index)
        cpu = None
        if not args.no_cpu_baseline and world == 1:              # (rank 0 at N = 1 only)
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle                                       # CPU baseline leg only
            o = pyoracle.OracleState()
            W.load_estimate(o, w)
            g = min(args.cpu_groups, args.groups)
            off = w.group_off[: g + 1]
            c0 = time.perf_counter()
            ro = o.estimate(w.table, off, w.pod_idx[: off[-1]], w.templates[:g], w.max_nodes, 0)
            cpu_s = time.perf_counter() - c0
            cev = int(ro.results["evals"].sum())
            cpu = {"value": cev / cpu_s, "unit": "evals/s", "cores": 1, "kind": "port",
                   "sample": f"oracle/casim_oracle.c Estimate of {g} of the {args.groups} C2 groups (one batch, "
                             f"{cev} evals in {cpu_s:.2f} s) on 1 thread of {cpu_model()}"}
        ms = elapsed / args.steps * 1e3
        result = {
            "metric": METRIC, "value": evals / elapsed, "unit": "evals/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "int64",
            "data": "synthetic: seeded C2 generator (autoscaler_amd/workloads.py), 64-shape pod catalog",
            "config": {
                "workload": "C2: heterogeneous pending pods x node-group templates, resource-fit only "
                            "(BASELINE.json configs[1]); one step = Estimate() for every group, every group's "
                            "node count and scheduled pods on the host",
                "pods": args.pods, "groups": args.groups, "existing_nodes": args.existing,
                "max_nodes_per_scaleup": args.max_nodes,
                "parallelism": f"the {args.groups} groups in {st['blocks']} contiguous blocks over {world} GPUs, "
                               "driven from one process through ca_multi_estimate_plan_run (one host thread per "
                               "device, replicated mirrors, lastIndex chain fixed up in the library)",
            },
            # the devices' kernels are not timed one by one here: the chain kernel's algorithmic
            # bytes over the whole step time (a lower bound of its rate)
            "roofline": {"bound": "hbm", "achieved": PHASE_BYTES["chain_ms"] * items / (ms / 1e3) / 1e9,
                         "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                         "frac": PHASE_BYTES["chain_ms"] * items / (ms / 1e3) / 1e9 / (HBM_PEAK_GBS * world),
                         "traffic": None, "kernel": "k_ffd_chain", "kernel_ms": None,
                         "bytes_per_unit": PHASE_BYTES["chain_ms"], "unit_of_work": "(pod, node group) item",
                         "units_per_launch": items, "basis": "step time over all devices (per-kernel times "
                                                             "are measured at N=1)"},
            "cpu_baseline": cpu,
            "extra": {
                "estimate_latency_ms": ms,
                "results_to_host": "32-bit pod ids in one page-locked buffer, each device's zero-copy publisher "
                                   "writing its block's slice",
                "blocks": st, "results_identical_to_1gpu": same, "items_per_step": items,
                "evals_per_step": evals / args.steps,
                "speedup_vs_cpu_baseline": (evals / elapsed) / cpu["value"] if cpu else None,
            },
        }
        print(json.dumps(result), flush=True)
        plan.close()
        multi.close()
        for m in mirrors:
            m.close()
    dist.barrier()
    dist.destroy_process_group()
    return result


def _free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def spawn_ranks(n: int) -> int:
    """--gpus N > 1 without a launcher: start N ranks under torch.distributed.run as a child
    process (nothing here has touched a GPU) and return its exit code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))         # --gpus is authoritative: N ranks, one per GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
              f"(torchrun --nproc-per-node {args.gpus} bench.py --gpus {args.gpus})", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # RCCL when every rank has a GPU of its own; with fewer GPUs than ranks (a rehearsal of
    # the N > 1 path on a one-GPU box) the ranks share devices round-robin and the collectives
    # run over gloo on host tensors (CASIM_BENCH_BACKEND overrides)
    shared = False
    if world > 1:
        import torch
        shared = torch.cuda.device_count() < world
    backend = os.environ.get("CASIM_BENCH_BACKEND", "gloo" if shared else "nccl")
    # N > 1: weak scaling by default — one Estimate batch of groups x N node groups, each
    # rank its own block of `groups` groups (rank 0's block is exactly the N = 1 workload),
    # the blocks chained through the checker's lastIndex by one all_gather of a 4-int record
    # per rank per step (shard.py).  CASIM_BENCH_SCALING=strong: the same 100 groups split
    # over the N GPUs (ca_multi_estimate_plan_run from rank 0, or CASIM_BENCH_MULTI=rccl).
    scaling = os.environ.get("CASIM_BENCH_SCALING", "weak") if world > 1 else "weak"
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend != "nccl" or shared:
            local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dist.init_process_group(backend)          # "nccl" is RCCL on ROCm
        if scaling == "strong" and os.environ.get("CASIM_BENCH_MULTI", "capi") != "rccl":
            return multi_main(args, world, rank, dist, f"cuda:{local}" if backend == "nccl" else "cpu")

    from autoscaler_amd import native, shard
    from autoscaler_amd import workloads as W

    # every rank holds the same cluster (the mirror is replicated) and runs its contiguous
    # block of the batch's node groups; the blocks are chained through the checker's
    # lastIndex (autoscaler_amd/shard.py).  Weak scaling: the batch has
    # groups x N groups (the generator draws group templates in order, so its first
    # `groups` groups are the N = 1 batch) and rank r runs groups [r*groups, (r+1)*groups);
    # strong scaling (rccl): the same `groups` groups in N blocks balanced by items.
    n_groups_total = args.groups * world if scaling == "weak" else args.groups
    w = W.c2(n_pods=args.pods, n_groups=n_groups_total, n_existing=args.existing, max_nodes=args.max_nodes, seed=42)
    if scaling == "weak":
        blocks = [args.groups * r for r in range(world + 1)]
    else:
        blocks = split_groups(w.group_off, world)
    g0, g1 = blocks[rank], blocks[rank + 1]
    off_blk = (w.group_off[g0:g1 + 1] - w.group_off[g0]).astype(np.int32)
    idx_blk = w.pod_idx[w.group_off[g0]:w.group_off[g1]]
    tm_blk = w.templates[g0:g1]
    mirror = native.Mirror(local)
    W.load_estimate(mirror, w)
    plan = native.EstimatePlan(mirror, w.table, off_blk, idx_blk, tm_blk)
    L0 = 0
    items = int(w.group_off[-1])                                # (pod, group) items of the whole batch
    items_blk = int(off_blk[-1])

    # results on the host as 16-bit podset indices when the podset allows it (C2: 50k pods;
    # ca_estimate_plan_run_u16, half the PCIe bytes), else 32-bit pod ids
    host_mode = "u16" if (len(w.table) <= 65535 and not args.with_nodes) else "i32"

    def run_block(lin, mode="host"):
        """This rank's block: results to the caller's page-locked buffer (headline: `host_mode`;
        "i32": 32-bit ids), or left in HBM ("device": extra.device_resident)."""
        if g1 == g0:
            return None, lin, 0, 0
        if mode == "host":
            mode = host_mode
        if args.with_nodes:
            out = plan.run(w.max_nodes, lin, want_nodes=True, copy=False)
        elif mode == "device":
            out = plan.run(w.max_nodes, lin, copy=False, device_results=True)
        elif mode == "u16":
            out = plan.run_u16(w.max_nodes, lin, copy=False)
        else:
            out = plan.run(w.max_nodes, lin, want_nodes=False, copy=False)
        # (lastIndex sensitivity: only the cross-rank chain of shard.run_sharded reads it)
        sens, succ = plan.chain_info() if dist is not None else (0, 0)
        return out, out.last_index, sens, succ

    coll_dev = f"cuda:{local}" if backend == "nccl" else "cpu"
    gather = shard.torch_all_gather(dist, coll_dev) if dist is not None else None

    def step(mode="host"):
        """One Estimate batch: this rank's block + the lastIndex chain across ranks."""
        run = (lambda lin: run_block(lin, mode))
        if dist is None:
            return run(L0)[0], 0
        out, _, extra = shard.run_sharded(run, L0, gather, rank)
        return out, extra

    def timed(mode):
        # the timed steps run without the library's per-phase timing events (8 event records
        # per step on the host's launch path); the phases come from the untimed steps below
        plan.set_phase_timing(False)
        for _ in range(args.warmup):
            step(mode)
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        evals, extras, out = 0, [], None
        for _ in range(args.steps):
            out, extra = step(mode)
            evals += int(out.results["evals"].sum()) if out is not None else 0
            extras.append(extra)
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        el = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([el, float(evals)], dtype=torch.float64, device=coll_dev)
            tmax, tsum = t.clone(), t.clone()
            dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
            dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
            return float(tmax[0]), int(tsum[1]), evals, extras, out
        return el, evals, evals, extras, out

    # headline: results on the host (Estimate latency = results on the host)
    elapsed, total_evals, evals, extras, hout = timed("host")
    host_pods = hout.sched_pod.copy() if hout is not None else None
    if host_pods is not None and host_pods.dtype == np.uint16:
        host_pods = np.where(host_pods == 0xFFFF, -1, host_pods.astype(np.int32))
    # per-phase device times: the same steps again, untimed
    chain_ms, sort_ms, rounds, phases, pub = [], [], [], [], []
    plan.set_phase_timing(True)
    for i in range(args.steps):
        step("host")
        st = plan.stats()
        chain_ms.append(st["chain_ms"] / max(st["rounds"], 1))
        sort_ms.append(st["sort_ms"])
        rounds.append(st["rounds"] + extras[i])
        ph = dict(st["phases"])
        ph["chain_ms"] = ph["chain_ms"] / max(st["rounds"], 1)       # one launch
        phases.append(ph)
        pub.append(st["results_path"])
    # device-resident variant (results left in HBM): the previous round's headline
    d_el, d_total, _, _, _ = timed("device")
    same = bool(host_pods is None or np.array_equal(host_pods, plan.fetch()))
    # 32-bit pod ids on the host (the previous round's headline), when the headline is u16
    host_i32 = None
    if host_mode == "u16":
        i_el, i_total, _, _, iout = timed("i32")
        host_i32 = {"ms_per_step": i_el / args.steps * 1e3, "evals_per_s": i_total / i_el,
                    "results_identical_to_headline": bool(iout is None or np.array_equal(host_pods, iout.sched_pod)),
                    "results": "scheduled pods as 32-bit pod ids in the caller's page-locked buffer "
                               "(ca_estimate_plan_run, zero-copy publisher)"}
    device_resident = {"ms_per_step": d_el / args.steps * 1e3, "evals_per_s": d_total / d_el,
                       "results_identical_to_host_mode": same,
                       "results": "scheduled pods left in HBM (ca_estimate_plan_run with sched_pod = NULL); "
                                  "results[] and lastIndex on the host"}
    # cold latency: a caller whose pending set changed since the last loop builds a new plan
    # (plan_prepare walks the batch's items on the host, checks float64 ties, uploads the
    # lists) and runs it once; and the one-shot Mirror.estimate (plan + run + teardown)
    cold = None
    if dist is None and g1 > g0:
        cp, cr, cb = [], [], []
        for _ in range(3):
            t0 = time.perf_counter()
            with native.EstimatePlan(mirror, w.table, off_blk, idx_blk, tm_blk) as p2:
                t1 = time.perf_counter()
                if host_mode == "u16":
                    p2.run_u16(w.max_nodes, L0, copy=False)
                else:
                    p2.run(w.max_nodes, L0, want_nodes=False, copy=False)
                t2 = time.perf_counter()
            cp.append(t1 - t0)
            cr.append(t2 - t1)
            t3 = time.perf_counter()
            mirror.estimate(w.table, off_blk, idx_blk, tm_blk, w.max_nodes, L0, want_nodes=False)
            cb.append(time.perf_counter() - t3)
        cold = {"plan_create_ms": float(np.median(cp) * 1e3), "first_run_ms": float(np.median(cr) * 1e3),
                "plan_create_plus_first_run_ms": float(np.median(np.add(cp, cr)) * 1e3),
                "one_shot_estimate_ms": float(np.median(cb) * 1e3),
                "note": "median of 3 on the headline's mirror: a new EstimatePlan over the same C2 batch (host item "
                        "walk, tie check, list upload) and its first run with results on the host as the headline; "
                        "one_shot = Mirror.estimate (plan + run + teardown, 32-bit ids copied to the host)"}
    n_cls = len(set(zip(w.table.pods["score_milli_cpu"].tolist(), w.table.pods["score_memory"].tolist())))
    n_merge = 1 if n_cls <= 256 else 2                            # radix passes (8-bit digits)
    ph_mean = {k: float(np.mean([p[k] for p in phases])) for k in phases[0]} if g1 > g0 else {}
    dom = max(PHASE_BYTES, key=lambda k: ph_mean.get(k, 0.0))
    per_item = PHASE_BYTES[dom] * (n_merge if dom == "merge_ms" else 1)
    kernel_ms = ph_mean.get(dom, 0.0)
    achieved = per_item * items_blk / (kernel_ms / 1e3) / 1e9 if kernel_ms > 0 else 0.0
    traffic, traffic_src = None, None
    tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")      # rocprofv3 --pmc passes (scripts/pmc_step.py)
    if os.path.exists(tf) and world == 1:
        with open(tf) as f:
            tj = json.load(f)
        for name in PHASE_KERNEL[dom].split("+")[:1]:
            rec = tj.get("kernels", {}).get(f"casim::{name}")
            if rec:
                traffic = rec.get("traffic_bytes_per_step", rec["traffic_bytes_per_launch"])
                traffic_src = f"profiles/pmc_traffic.json ({tj.get('source', '')})"

    # N > 1: configs 3-5 beside the C2 line, every rank taking part (one block each)
    multi_legs = {}
    if dist is not None:
        ctx = RankCtx(dist, rank, world, local, coll_dev, shared)
        if not args.no_sweep:
            multi_legs["c3_multi"] = c3_multi_leg(args, ctx)
        if not args.no_c4:
            multi_legs["c4_multi"] = c4_multi_leg(args, ctx)
        if not args.no_runonce:
            multi_legs["c5_runonce_multi"] = c5_multi_leg(args, ctx)

    result = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:              # (rank 0 at N = 1 only)
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle                                       # CPU baseline leg only
            o = pyoracle.OracleState()
            W.load_estimate(o, w)
            g = min(args.cpu_groups, args.groups)
            off = w.group_off[: g + 1]
            c0 = time.perf_counter()
            ro = o.estimate(w.table, off, w.pod_idx[: off[-1]], w.templates[:g], w.max_nodes, L0)
            cpu_s = time.perf_counter() - c0
            cpu_evals = int(ro.results["evals"].sum())
            cpu = {"value": cpu_evals / cpu_s, "unit": "evals/s", "cores": 1, "kind": "port",
                   "sample": f"oracle/casim_oracle.c Estimate of {g} of the {args.groups} C2 groups (one batch, "
                             f"{cpu_evals} evals in {cpu_s:.2f} s) on 1 thread of {cpu_model()}",
                   "estimate_ms": cpu_s * 1e3}
        ms = elapsed / args.steps * 1e3
        result = {
            "metric": METRIC,
            "value": total_evals / elapsed,
            "unit": "evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic: seeded C2 generator (autoscaler_amd/workloads.py), 64-shape pod catalog",
            "config": {
                "workload": "C2: heterogeneous pending pods x node-group templates, resource-fit only "
                            "(BASELINE.json configs[1]); one step = Estimate() for every group, every group's "
                            "node count and scheduled pods on the host",
                "pods": args.pods, "groups": n_groups_total, "groups_per_gpu": g1 - g0,
                "existing_nodes": args.existing,
                "max_nodes_per_scaleup": args.max_nodes,
                "parallelism": (f"{n_groups_total} groups = {args.groups} per GPU x {world} GPU(s) (weak scaling), "
                                if scaling == "weak" else f"the {args.groups} groups in {world} contiguous blocks, ")
                               + "one block per GPU (one process each), lastIndex chained by an all_gather of a "
                                 "4-int record per rank per step",
            },
            "roofline": {
                "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                "traffic_unit": "HBM bytes per step of the phase (all its launches)",
                "traffic_source": traffic_src,
                "kernel": PHASE_KERNEL[dom], "kernel_ms": kernel_ms,
                "bytes_per_unit": per_item, "unit_of_work": "(pod, node group) item",
                "units_per_launch": items_blk,
            },
            "cpu_baseline": cpu,
            "extra": {
                "estimate_latency_ms": ms,
                "results_to_host": "zero-copy publisher kernel on a second stream writes each final chunk of 4096 "
                                   "scheduled pods into the caller's page-locked buffer while the chains run, as "
                                   + ("16-bit podset indices (ca_estimate_plan_run_u16, "
                                      if host_mode == "u16" else "32-bit pod ids (ca_estimate_plan_run, ")
                                   + f"{(2 if host_mode == 'u16' else 4) * items} B per step); results path per step: "
                                   f"{sorted(set(pub)) if pub else None}",
                "device_resident": device_resident,
                "host_int32_ids": host_i32,
                "cold": cold,
                "sort_ms": float(np.mean(sort_ms)) if sort_ms else None,
                "phases_ms": ph_mean,
                "chain_kernel_ms": ph_mean.get("chain_ms"),
                "items_per_s": items * args.steps / elapsed,
                "eval_equivalent_GBps": (BYTES_PER_EVAL * (evals / args.steps) / (ph_mean["chain_ms"] / 1e3) / 1e9
                                         if ph_mean.get("chain_ms") else None),
                "speculation_rounds": float(np.mean(rounds)) if rounds else None,
                "evals_per_step": total_evals / args.steps,
                "rank0_groups": [g0, g1],
                "speedup_vs_cpu_baseline": (total_evals / elapsed) / cpu["value"] if cpu else None,
            },
        }
        result["extra"].update(multi_legs)
        if shared:
            result["config"]["devices"] = f"{world} ranks sharing {torch.cuda.device_count()} GPU(s): a rehearsal " \
                                          "of the N-GPU launch (gloo collectives), not an N-GPU measurement"
        if world == 1 and not args.no_sweep:
            result["extra"]["sweep"] = sweep_leg(args, local, not args.no_cpu_baseline)
        if world == 1 and not args.no_c4:
            result["extra"]["c4"] = c4_leg(args, local, not args.no_cpu_baseline)
        if world == 1 and not args.no_unlimited:
            result["extra"]["c2_unlimited"] = c2_unlimited_leg(args, local, not args.no_cpu_baseline)
        if world == 1 and not args.no_expansion:
            result["extra"]["expansion"] = expansion_leg(args, local, not args.no_cpu_baseline)
        if world == 1 and not args.no_filter:
            result["extra"]["filter"] = filter_leg(args, local, not args.no_cpu_baseline)
        if world == 1 and not args.no_util:
            result["extra"]["utilization"] = utilization_leg(args, local, not args.no_cpu_baseline)
        if world == 1 and not args.no_runonce:
            result["extra"]["c5_runonce"] = runonce_leg(args, local, not args.no_cpu_baseline)
        if world == 1 and not args.no_planner:
            result["extra"]["planner"] = planner_leg(args, local, not args.no_cpu_baseline)
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    plan.close()
    mirror.close()
    return result


if __name__ == "__main__":
    main()
