"""Scale-down planner over the mirror (CA/core/scaledown/planner/planner.go, --parallel-drain).

The host half of the planner: recently evicted pods injected into a fork of the snapshot
(injectRecentlyEvictedPods, :198-234), the eligibility split, the unneeded-nodes limit
(:296-334) and the PDB tracker (CA/core/scaledown/pdb/basic.go).  The candidate loop
itself (categorizeNodes, :252-296) is one ca_plan_removals call through
RemovalSimulator(persist_successful_simulations=True).SimulateNodeRemovals, which commits
every removable candidate into the fork; UpdateClusterState reverts the fork afterwards
(:108-110), as the reference does.
"""
from __future__ import annotations

import copy
from typing import Callable, Optional

from .clustersnapshot import ClusterSnapshot
from .drain import ListerRegistry, NodeDeleteOptions, NotEnoughPdb, BlockingPod, is_mirror_pod, pdb_matches
from .k8s import Pod, is_daemonset_pod
from .predicatechecker import SchedulerBasedPredicateChecker
from .simulator import HintingSimulator, RemovalSimulator, UnexpectedError, UnremovableNode

ConfigSourceAnnotationKey = "kubernetes.io/config.source"
ApiserverSource = "api"


class RemainingPdbTracker:
    """basicRemainingPdbTracker (CA/core/scaledown/pdb/basic.go:33-101)."""

    def __init__(self):
        self.pdbs: list = []

    def SetPdbs(self, pdbs: list) -> None:  # noqa: N802
        self.pdbs = [copy.deepcopy(p) for p in pdbs]

    def GetPdbs(self) -> list:  # noqa: N802
        return self.pdbs

    def CanRemovePods(self, pods: list):  # noqa: N802
        in_parallel, blocking = True, None
        for pdb in self.pdbs:
            count = 0
            for pod in pods:
                if pdb_matches(pdb, pod):
                    count += 1
                    if pdb.disruptions_allowed < 1:
                        return False, False, BlockingPod(pod, NotEnoughPdb)
                    if pdb.disruptions_allowed < count:
                        in_parallel, blocking = False, BlockingPod(pod, NotEnoughPdb)
        return True, in_parallel, blocking

    def RemovePods(self, pods: list) -> None:  # noqa: N802
        for pdb in self.pdbs:
            for pod in pods:
                if pdb_matches(pdb, pod):
                    pdb.disruptions_allowed -= 1

    def Clear(self) -> None:  # noqa: N802
        self.pdbs = []


def is_static_pod(pod: Pod) -> bool:
    """pod_util.IsStaticPod (CA/utils/pod/pod.go:55-62)."""
    src = pod.annotations.get(ConfigSourceAnnotationKey)
    return src is not None and src != ApiserverSource


def filter_recreatable_pods(pods: list) -> list:
    """pod_util.FilterRecreatablePods (CA/utils/pod/pod.go:65-74)."""
    return [p for p in pods if not (is_static_pod(p) or is_mirror_pod(p) or is_daemonset_pod(p))]


KNOWN_OWNERS = ("StatefulSet", "Job", "ReplicaSet", "ReplicationController")


def filter_out_recreated_pods(pods: list, replicas: Callable) -> list:
    """filterOutRecreatedPods (planner.go:209-233).  replicas(owner_ref, namespace) returns
    (target, current) replicas of the controller, or None when it is unknown (error)."""
    out, added = [], {}
    for pod in pods:
        ref = next((r for r in pod.owner_refs if r.kind in KNOWN_OWNERS), None)   # getKnownOwnerRef
        if ref is None:
            out.append(pod)
            continue
        rep = replicas(ref, pod.namespace)
        if rep is None:
            out.append(pod)
            continue
        target, current = rep
        if target > current and added.get(ref.uid, 0) < target - current:
            out.append(pod)
            added[ref.uid] = added.get(ref.uid, 0) + 1
    return out


class Planner:
    """planner.Planner (planner.go:60-100): UpdateClusterState keeps the unneeded and
    unremovable node sets; the simulation runs on the device."""

    def __init__(self, snapshot: ClusterSnapshot, predicate_checker: SchedulerBasedPredicateChecker,
                 delete_options: NodeDeleteOptions = NodeDeleteOptions(), listers: Optional[ListerRegistry] = None,
                 max_scale_down_parallelism: int = 10, scale_down_unneeded_time: float = 600.0,
                 eligible: Optional[Callable] = None, replicas: Optional[Callable] = None, pdbs: Optional[list] = None):
        self.snapshot = snapshot
        self.rs = RemovalSimulator(listers, snapshot, predicate_checker, delete_options=delete_options,
                                   persist_successful_simulations=True)
        self.actuation_injector = HintingSimulator(predicate_checker)
        self.max_parallelism = max_scale_down_parallelism
        self.unneeded_time = scale_down_unneeded_time
        self.eligible = eligible                   # FilterOutUnremovable stand-in: names -> eligible names
        self.replicas = replicas or (lambda ref, ns: None)
        self.pdb_tracker = RemainingPdbTracker()
        self.pdb_tracker.SetPdbs(pdbs or [])
        self.latest_update: Optional[float] = None
        self.min_update_interval = scale_down_unneeded_time if scale_down_unneeded_time > 0 else 1e-9   # New (:80-83)
        self.unneeded: dict = {}                  # name -> NodeToBeRemoved
        self.unremovable: dict = {}               # name -> UnremovableNode
        self.inject_error: Optional[str] = None

    def unneeded_nodes_limit(self) -> int:
        """unneededNodesLimit (planner.go:318-334), durations in integer nanoseconds."""
        n = self.max_parallelism
        limit = len(self.unneeded) + 2 * n
        loop = max(int(round(self.min_update_interval * 1e9)), 1)
        u = max(int(round(self.unneeded_time * 1e9)), loop)
        return min(n * (u // loop) + n, limit)

    def UpdateClusterState(self, pod_destinations: list, scale_down_candidates: list,  # noqa: N802
                           recent_evictions: list = (), current_time: float = 0.0,
                           deletions_in_progress: tuple = ()) -> None:
        """planner.go:103-126: fork, inject, categorize, revert."""
        if self.latest_update is not None:                       # :104-107
            self.min_update_interval = min(self.min_update_interval, current_time - self.latest_update)
        self.latest_update = current_time
        snap = self.snapshot
        snap.Fork()
        try:
            self.inject_error = self._inject(filter_out_recreated_pods(filter_recreatable_pods(list(recent_evictions)),
                                                                       self.replicas))
            gone = set(deletions_in_progress)
            dests = [n for n in pod_destinations if n not in gone]
            cands = [n for n in scale_down_candidates if n not in gone]
            self._categorize(dests, cands)
        finally:
            snap.Revert()
        self.rs.DropOldHints()
        self.actuation_injector.DropOldHints()

    def _inject(self, pods: list) -> Optional[str]:
        """injectPods (planner.go:236-248): TrySchedulePods(ScheduleAnywhere, breakOnFailure)."""
        pods = [copy.copy(p) for p in pods]
        for p in pods:                                           # ClearPodNodeNames (pod.go:77-85)
            p.node_name = ""
        statuses, _, err = self.actuation_injector.TrySchedulePods(self.snapshot, pods, None, True)
        if err is not None:
            return str(err)
        if len(statuses) != len(pods):
            return f"can reschedule only {len(statuses)} out of {len(pods)} pods from ongoing deletions"
        return None

    def _categorize(self, destinations: list, candidates: list) -> None:
        """categorizeNodes (planner.go:252-296), the loop on the device."""
        self.unremovable = {}
        names = list(candidates)
        if self.eligible is not None:
            ok = set(self.eligible(names))
            for n in names:
                if n not in ok:
                    self.unremovable[n] = UnremovableNode(self.snapshot.Get(n).node, UnexpectedError)
            names = [n for n in names if n in ok]
        removable, unremovable = self.rs.SimulateNodeRemovals(names, destinations, self.latest_update or 0.0,
                                                              self.pdb_tracker, self.unneeded_nodes_limit())
        for u in unremovable:
            self.unremovable[u.node.name] = u
        self.unneeded = {r.node.name: r for r in removable}      # unneededNodes.Update (:288)

    def UnneededNodes(self) -> list:  # noqa: N802
        return list(self.unneeded)

    def UnremovableNodes(self) -> list:  # noqa: N802
        return list(self.unremovable.values())
