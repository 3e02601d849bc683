"""FilterOutSchedulable pod list processor (CA/core/podlistprocessor/filter_out_schedulable.go).

``filterOutSchedulableByPacking`` (:95-124) sorts the pending pods by priority, runs
HintingSimulator.TrySchedulePods(snapshot, pods, ScheduleAnywhere, breakOnFailure=false)
on the unforked snapshot (so every pod that fits stays placed) and returns the pods
that still do not fit.  Here the whole TrySchedulePods loop is one device call
(``ca_filter_out_schedulable``, autoscaler_amd/csrc/filter.hip); the host keeps the
pod-key hints (hints.go) and the SimilarPodsScheduling keys (controller UID + labels +
spec, similar_pods.go:43-111) as class ids with their controllers.
"""
from __future__ import annotations

import numpy as np

from .clustersnapshot import ClusterSnapshot
from .gosort import sort_slice_desc
from .k8s import Pod
from .predicatechecker import SchedulerBasedPredicateChecker, unsupported
from .simulator import HintingSimulator, Hints, Status


def PodPriority(pod: Pod) -> int:  # noqa: N802 - corev1helpers.PodPriority
    return 0 if pod.priority is None else int(pod.priority)


def TrySchedulePodsAnywhere(sim: HintingSimulator, snapshot: ClusterSnapshot, pods: list):  # noqa: N802
    """HintingSimulator.TrySchedulePods(snapshot, pods, ScheduleAnywhere, false)
    (hinting_simulator.go:58-89) as one batched call; returns (statuses, overflowing)."""
    if not pods:
        return [], 0
    table = snapshot.encode(pods)
    n_classes = int(table.pods["similar_class"].max()) + 1
    owners = snapshot.interner.class_owners(max(n_classes, 0))
    hints = np.full(len(pods), -1, np.int32)
    for k, pod in enumerate(pods):
        name, ok = sim.hints.Get(Hints.key(pod))
        if ok and name in snapshot._state.pos:
            hints[k] = snapshot.position(name)
    pc = sim.predicate_checker
    with unsupported("FilterOutSchedulable: a pending pod or the snapshot is out of kernel scope"):
        out = snapshot.backend.filter_out_schedulable(table, None, owners if n_classes > 0 else None, hints,
                                                      pc.last_index)
    pc.last_index = out.last_index
    pc.evals += int(out.evals)
    statuses, placed = [], []
    for k, pod in enumerate(pods):
        node = int(out.node[k])
        if node < 0:
            continue
        name = snapshot.name_at(node)
        sim.hints.Set(Hints.key(pod), name)                   # hinting_simulator.go:95 / :123
        statuses.append(Status(pod, name))
        placed.append((pod, name, int(out.pod_id[k])))
    snapshot.record_added_pods(placed)
    return statuses, int(out.n_overflowing)


class FilterOutSchedulablePodListProcessor:
    """filterOutSchedulablePodListProcessor (filter_out_schedulable.go:33-47)."""

    def __init__(self, predicate_checker: SchedulerBasedPredicateChecker, simulator: HintingSimulator = None):
        self.schedulingSimulator = simulator or HintingSimulator(predicate_checker)
        self.overflowing_controllers = 0          # metrics.UpdateOverflowingControllers

    def Process(self, snapshot: ClusterSnapshot, unschedulable_pods: list) -> list:  # noqa: N802
        return self.filterOutSchedulableByPacking(unschedulable_pods, snapshot)

    def filterOutSchedulableByPacking(self, unschedulable_candidates: list,  # noqa: N802
                                      snapshot: ClusterSnapshot) -> list:
        # :97-99 sort.Slice by priority, descending: Go 1.19's pdqsort, ties included (gosort.py)
        perm = sort_slice_desc([PodPriority(p) for p in unschedulable_candidates])
        unschedulable_candidates[:] = [unschedulable_candidates[i] for i in perm]
        statuses, overflow = TrySchedulePodsAnywhere(self.schedulingSimulator, snapshot, unschedulable_candidates)
        scheduled = {id(s.pod) for s in statuses}
        still = [p for p in unschedulable_candidates if id(p) not in scheduled]      # :111-116
        self.overflowing_controllers = overflow
        self.schedulingSimulator.DropOldHints()                                       # :121
        return still

    def CleanUp(self) -> None:  # noqa: N802
        pass


def NewFilterOutSchedulablePodListProcessor(predicate_checker):  # noqa: N802
    return FilterOutSchedulablePodListProcessor(predicate_checker)
