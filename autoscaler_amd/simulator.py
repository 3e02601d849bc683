"""RemovalSimulator over the mirror (CA/simulator/cluster.go, CA/simulator/scheduling).

FindNodesToRemove(candidates, destinations, timestamp, pdbs) runs the legacy
(canPersist=false) sweep on the device in one call: the host applies the drain
policy (GetPodsToMove) per candidate and passes the verdicts, the pods to move and
the hints (pod UID -> node) across the C ABI.  HintingSimulator keeps Hints with
the current/old generations of hints.go:29-72.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import abi
from .clustersnapshot import ClusterSnapshot
from .drain import BlockingPod, ListerRegistry, NodeDeleteOptions, get_pods_to_move
from .k8s import Node, Pod, is_daemonset_pod
from .predicatechecker import SchedulerBasedPredicateChecker, unsupported
from .scope import UnsupportedByKernels, out_of_scope_reason

# UnremovableReason (cluster.go:58-90)
(NoReason, ScaleDownDisabledAnnotation, ScaleDownUnreadyDisabled, NotAutoscaled, NotUnneededLongEnough,
 NotUnreadyLongEnough, NodeGroupMinSizeReached, MinimalResourceLimitExceeded, CurrentlyBeingDeleted,
 NotUnderutilized, NotUnneededOtherReason, RecentlyUnremovable, NoPlaceToMovePods, BlockedByPod,
 UnexpectedError) = range(15)


@dataclass
class NodeToBeRemoved:
    node: Node
    pods_to_reschedule: list = field(default_factory=list)
    daemonset_pods: list = field(default_factory=list)
    is_risky: bool = False


@dataclass
class UnremovableNode:
    node: Node
    reason: int
    blocking_pod: Optional[BlockingPod] = None


class Hints:
    """scheduling.Hints (hints.go:29-72): pod key -> node name, two generations."""

    def __init__(self):
        self.current: dict = {}
        self.old: dict = {}

    @staticmethod
    def key(pod: Pod) -> str:                       # HintKeyFromPod (hints.go:31-37)
        return pod.uid if pod.uid else f"{pod.namespace}/{pod.name}"

    def Get(self, key: str):  # noqa: N802
        if key in self.current:
            return self.current[key], True
        if key in self.old:
            return self.old[key], True
        return "", False

    def Set(self, key: str, node: str) -> None:  # noqa: N802
        self.current[key] = node

    def DropOld(self) -> None:  # noqa: N802
        self.old = self.current
        self.current = {}


@dataclass
class Status:
    """scheduling.Status (hinting_simulator.go:30-34)."""
    pod: Pod
    node_name: str


class SimilarPodsScheduling:
    """similar_pods.go:43-111: unschedulable controller-equivalent pods seen in one call."""

    max_pods_per_owner_ref = 10

    def __init__(self):
        self.items: dict = {}
        self.overflowing: set = set()

    @staticmethod
    def _key(pod: Pod):
        ref = pod.controller_ref()
        return None if ref is None else ref.uid

    @staticmethod
    def _sig(pod: Pod):
        return (repr(sorted(pod.labels.items())), repr((pod.containers, pod.init_containers, pod.overhead,
                                                        pod.node_selector, pod.affinity, pod.tolerations,
                                                        pod.volumes, pod.topology_spread,
                                                        pod.node_name, pod.priority)))

    def IsSimilarUnschedulable(self, pod: Pod) -> bool:  # noqa: N802
        k = self._key(pod)
        return k is not None and self._sig(pod) in self.items.get(k, [])

    def SetUnschedulable(self, pod: Pod) -> None:  # noqa: N802
        k = self._key(pod)
        if k is None or is_daemonset_pod(pod):           # similar_pods.go:86-88
            return
        lst = self.items.setdefault(k, [])
        if len(lst) >= self.max_pods_per_owner_ref:
            self.overflowing.add(k)
            return
        lst.append(self._sig(pod))


class HintingSimulator:
    """scheduling.HintingSimulator (hinting_simulator.go:36-135) composed from the
    predicate-checker entry points (one device call per pod: the compatibility path)."""

    def __init__(self, predicate_checker: SchedulerBasedPredicateChecker):
        self.predicate_checker = predicate_checker
        self.hints = Hints()

    def TrySchedulePods(self, snapshot: ClusterSnapshot, pods: list, is_node_acceptable=None,  # noqa: N802
                        break_on_failure: bool = False):
        similar = SimilarPodsScheduling()
        statuses = []
        pc = self.predicate_checker
        for pod in pods:
            node_name = ""
            hk = Hints.key(pod)
            hinted, ok = self.hints.Get(hk)                            # findNodeWithHints (:91-108)
            if ok and pc.CheckPredicates(snapshot, pod, hinted) is None:
                self.hints.Set(hk, hinted)
                info = snapshot.Get(hinted)
                if is_node_acceptable is None or is_node_acceptable(info):
                    node_name = hinted
            if not node_name:                                          # findNode (:110-125)
                if not similar.IsSimilarUnschedulable(pod):
                    name, err = pc.FitsAnyNodeMatching(snapshot, pod, is_node_acceptable)
                    if err is not None:
                        similar.SetUnschedulable(pod)
                    else:
                        self.hints.Set(hk, name)
                        node_name = name
            if node_name:
                snapshot.AddPod(pod, node_name)
                statuses.append(Status(pod, node_name))
            elif break_on_failure:
                break
        return statuses, len(similar.overflowing), None

    def DropOldHints(self) -> None:  # noqa: N802
        self.hints.DropOld()


class RemovalSimulator:
    def __init__(self, listers: Optional[ListerRegistry], cluster_snapshot: ClusterSnapshot,
                 predicate_checker: SchedulerBasedPredicateChecker, usage_tracker=None,
                 delete_options: NodeDeleteOptions = NodeDeleteOptions(), persist_successful_simulations: bool = False):
        if persist_successful_simulations:
            raise NotImplementedError("canPersist=true (planner) is sequential and committing: DESIGN.md §next")
        self.listers = listers
        self.cluster_snapshot = cluster_snapshot
        self.predicate_checker = predicate_checker
        self.delete_options = delete_options
        self.hints = Hints()
        self.last_stats = None

    def FindNodesToRemove(self, candidates: list, destinations: list, timestamp: float = 0.0,  # noqa: N802
                          pdbs: Optional[list] = None):
        snap = self.cluster_snapshot
        pdbs = pdbs or []
        names = snap.node_names()
        dest_set = set(destinations)
        mask = np.array([n in dest_set for n in names], np.uint8)
        cand_pos, status, move_off, move_ids, moved_pods, ds_pods, blocking = [], [], [0], [], [], [], []
        for name in candidates:
            info = snap.Get(name)
            pos = snap.position(name)
            cand_pos.append(pos)
            st = 0
            pods_to_move, ds, block = [], [], None
            if name not in dest_set:                                   # cluster.go:157-160
                st = abi.CA_UNREMOVABLE_UNEXPECTED_ERROR
            else:
                pods_to_move, ds, block, err = get_pods_to_move(info.pods, self.delete_options, self.listers, pdbs,
                                                                timestamp)
                if err is not None:
                    st = abi.CA_UNREMOVABLE_BLOCKED_BY_POD if block is not None else abi.CA_UNREMOVABLE_UNEXPECTED_ERROR
            status.append(st)
            moved_pods.append(pods_to_move if st == 0 else [])
            ds_pods.append(ds)
            blocking.append(block)
            if st == 0:
                ids = {id(p): pid for p, pid in snap.pod_ids(name)}
                move_ids.extend(ids[id(p)] for p in pods_to_move)
            move_off.append(len(move_ids))
        # Hints.Get per mirror pod id
        n_ids = max([pid for n in names for _, pid in snap.pod_ids(n)] + [-1]) + 1
        hints = np.full(max(n_ids, 1), -1, np.int32)
        id_to_pod = {pid: p for n in names for p, pid in snap.pod_ids(n)}
        for pid, p in id_to_pod.items():
            node, ok = self.hints.Get(Hints.key(p))
            if ok and node in snap._state.pos:
                hints[pid] = snap.position(node)
        before = hints.copy()
        with unsupported("FindNodesToRemove: the snapshot holds a pod with required anti-affinity"):
            out = snap.backend.find_nodes_to_remove(np.array(cand_pos, np.int32), mask, np.array(status, np.int32),
                                                    np.array(move_off, np.int32), np.array(move_ids, np.int32), hints,
                                                    self.predicate_checker.last_index)
        cut = next((c for c in range(len(candidates))
                    if int(out.results[c]["reason"]) == abi.CA_UNREMOVABLE_OUT_OF_SCOPE), None)
        if cut is not None:
            why = next((out_of_scope_reason(p) for p in moved_pods[cut] if out_of_scope_reason(p)), "out of scope")
            raise UnsupportedByKernels(f"FindNodesToRemove: candidate {candidates[cut]}: {why}")
        self.predicate_checker.last_index = out.last_index
        self.predicate_checker.evals += int(out.results["evals"].sum())
        for pid in np.nonzero(out.hints != before)[0]:
            self.hints.Set(Hints.key(id_to_pod[int(pid)]), names[int(out.hints[pid])])
        for i, mid in enumerate(move_ids):                # a re-set to the same node is a Set too
            d = out.dest[i]
            if d >= 0:
                self.hints.Set(Hints.key(id_to_pod[mid]), names[int(d)])
        to_remove, unremovable = [], []
        for c, name in enumerate(candidates):
            node = snap.Get(name).node
            r = out.results[c]
            if int(r["removable"]):
                to_remove.append(NodeToBeRemoved(node, list(moved_pods[c]), list(ds_pods[c])))
            else:
                reason = int(r["reason"])
                unremovable.append(UnremovableNode(node, reason, blocking[c] if reason == BlockedByPod else None))
        self.last_stats = out
        return to_remove, unremovable

    def FindEmptyNodesToRemove(self, candidates: list, timestamp: float = 0.0) -> list:  # noqa: N802
        """cluster.go:187-202: GetPodsToMove with nil listers; empty iff no error and nothing to move."""
        out = []
        for name in candidates:
            try:
                info = self.cluster_snapshot.Get(name)
            except KeyError:
                continue
            pods, _, _, err = get_pods_to_move(info.pods, self.delete_options, None, [], timestamp)
            if err is None and not pods:
                out.append(name)
        return out

    def DropOldHints(self) -> None:  # noqa: N802
        self.hints.DropOld()


def NewRemovalSimulator(listers, cluster_snapshot, predicate_checker, usage_tracker=None,  # noqa: N802
                        delete_options=NodeDeleteOptions(), persist=False):
    return RemovalSimulator(listers, cluster_snapshot, predicate_checker, usage_tracker, delete_options, persist)
