"""RemovalSimulator over the mirror (CA/simulator/cluster.go, CA/simulator/scheduling).

FindNodesToRemove(candidates, destinations, timestamp, pdbs) runs the legacy
(canPersist=false) sweep on the device in one call: the host applies the drain
policy (GetPodsToMove) per candidate and passes the verdicts, the pods to move and
the hints (pod UID -> node) across the C ABI.  HintingSimulator keeps Hints with
the current/old generations of hints.go:29-72.

With persist_successful_simulations=True (the planner, planner.go:89) every removable
candidate's simulation is committed: SimulateNodeRemovals runs the planner's candidate
loop (planner.go:261-285) in one ca_plan_removals call and records the committed moves
in the snapshot; SimulateNodeRemoval is the one-candidate case (cluster.go:145).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import abi
from .clustersnapshot import ClusterSnapshot
from .drain import BlockingPod, ListerRegistry, NodeDeleteOptions, NotEnoughPdb, get_pods_to_move, pdb_matches
from .intern import TPU_PREFIX
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


def moved_copy(pod: Pod) -> Pod:
    """The pod findPlaceFor schedules: a copy with Spec.NodeName cleared (cluster.go:235-240)
    and TPU requests cleared (tpu.ClearTPURequests, tpu.go:57-79, applied at cluster.go:225)."""
    q = dataclasses.replace(pod, node_name="")
    if any(k.startswith(TPU_PREFIX) for c in pod.containers for k in c.requests):
        q.containers = [dataclasses.replace(c, requests={k: v for k, v in c.requests.items()
                                                         if not k.startswith(TPU_PREFIX)})
                        for c in pod.containers]
    return q


class RemovalSimulator:
    def __init__(self, listers: Optional[ListerRegistry], cluster_snapshot: ClusterSnapshot,
                 predicate_checker: SchedulerBasedPredicateChecker, usage_tracker=None,
                 delete_options: NodeDeleteOptions = NodeDeleteOptions(), persist_successful_simulations: bool = False):
        self.can_persist = persist_successful_simulations
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

    def SimulateNodeRemovals(self, candidates: list, destinations, timestamp: float = 0.0,  # noqa: N802
                             pdb_tracker=None, limit: int = 0):
        """The planner's candidate loop (planner.go:261-285) with canPersist=true: each
        candidate is SimulateNodeRemoval'd on the snapshot the earlier ones committed into;
        a removable one leaves the destinations and its pods are charged to pdb_tracker
        (a RemainingPdbTracker).  Stops once `limit` (> 0) candidates are removable.
        Returns (removable [NodeToBeRemoved], unremovable [UnremovableNode]) in candidate
        order; skipped candidates are in neither."""
        if not self.can_persist:
            raise ValueError("SimulateNodeRemovals commits: build the simulator with persist_successful_simulations")
        snap = self.cluster_snapshot
        pdbs = pdb_tracker.GetPdbs() if pdb_tracker is not None else []
        names = snap.node_names()
        dest_set = set(destinations)
        mask = np.array([n in dest_set for n in names], np.uint8)
        cand_pos, status, move_off, move_ids, ds_pods, blocking = [], [], [0], [], [], []
        id_to_pod = {pid: p for n in names for p, pid in snap.pod_ids(n)}
        for name in candidates:
            cand_pos.append(snap.position(name))
            st, pods_to_move, ds, block = 0, [], [], None
            if name not in dest_set:                                   # cluster.go:157-160
                st = abi.CA_UNREMOVABLE_UNEXPECTED_ERROR
            else:
                pods_to_move, ds, block, err = get_pods_to_move(snap.Get(name).pods, self.delete_options,
                                                                self.listers, pdbs, timestamp, check_pdbs=False)
                if err is not None:
                    st = abi.CA_UNREMOVABLE_BLOCKED_BY_POD if block is not None else abi.CA_UNREMOVABLE_UNEXPECTED_ERROR
            status.append(st)
            ds_pods.append(ds)
            blocking.append(block)
            if st == 0:
                ids = {id(p): pid for p, pid in snap.pod_ids(name)}
                move_ids.extend(ids[id(p)] for p in pods_to_move)
            move_off.append(len(move_ids))
        n_ids = max(list(id_to_pod) + [-1]) + 1
        hints = np.full(n_ids, -1, np.int32)
        for pid, p in id_to_pod.items():
            node, ok = self.hints.Get(Hints.key(p))
            if ok and node in snap._state.pos:
                hints[pid] = snap.position(node)
        pdb_off, pdb_idx = [0], []
        for pid in range(n_ids):                       # RemainingPdbTracker memberships per pod
            p = id_to_pod.get(pid)
            if p is not None:
                pdb_idx.extend(k for k, b in enumerate(pdbs) if pdb_matches(b, p))
            pdb_off.append(len(pdb_idx))
        allowed = [b.disruptions_allowed for b in pdbs]
        before = hints.copy()
        with unsupported("SimulateNodeRemovals: the snapshot holds a pod with required anti-affinity"):
            out = snap.backend.plan_removals(np.array(cand_pos, np.int32), mask, np.array(status, np.int32),
                                             np.array(move_off, np.int32), np.array(move_ids, np.int32), hints,
                                             self.predicate_checker.last_index, limit, allowed,
                                             np.array(pdb_off, np.int32), np.array(pdb_idx, np.int32))
        # the commits: copies of the moved pods (ids in commit order), recorded in the snapshot
        pods_by_id = dict(id_to_pod)
        groups, resched = [], {}
        for mv in out.moves:
            c, pid, nid, dest = int(mv["candidate"]), int(mv["pod"]), int(mv["new_pod"]), int(mv["node"])
            pod = pods_by_id[pid]
            cp = moved_copy(pod)
            pods_by_id[nid] = cp
            if not groups or groups[-1][0] != c:
                groups.append((c, []))
            groups[-1][1].append((pod, cp, names[dest], nid))
            resched.setdefault(c, []).append(pod)
        snap.record_moves([(candidates[c], mv) for c, mv in groups])
        for k, b in enumerate(pdbs):                   # RemovePods (basic.go:86-95)
            b.disruptions_allowed = int(out.allowed[k])
        self.predicate_checker.last_index = out.last_index
        self.predicate_checker.evals += int(out.results["evals"].sum())
        for pid in np.nonzero(out.hints != before)[0]:
            self.hints.Set(Hints.key(id_to_pod[int(pid)]), names[int(out.hints[pid])])
        for c, mv in groups:                           # Hints.Set of every placement (a re-set is a Set)
            for pod, _, dest, _ in mv:
                self.hints.Set(Hints.key(pod), dest)
        to_remove, unremovable = [], []
        for c, name in enumerate(candidates):
            r = out.results[c]
            reason = int(r["reason"])
            if reason == abi.CA_UNREMOVABLE_OUT_OF_SCOPE:
                why = next((out_of_scope_reason(id_to_pod[i]) for i in move_ids[move_off[c]:move_off[c + 1]]
                            if out_of_scope_reason(id_to_pod[i])), "out of scope")
                raise UnsupportedByKernels(f"SimulateNodeRemovals: candidate {name}: {why}")
            if reason == abi.CA_UNREMOVABLE_NOT_RUN:
                continue
            node = snap.Get(name).node
            if int(r["removable"]):
                to_remove.append(NodeToBeRemoved(node, list(resched.get(c, [])), list(ds_pods[c]), bool(r["risky"])))
            else:
                bp = blocking[c] if reason == BlockedByPod else None
                if int(r["blocking_pod"]) >= 0:
                    bp = BlockingPod(pods_by_id[int(r["blocking_pod"])], NotEnoughPdb)
                unremovable.append(UnremovableNode(node, reason, bp))
        self.last_stats = out
        return to_remove, unremovable

    def SimulateNodeRemoval(self, node_name: str, destination_map, timestamp: float = 0.0,  # noqa: N802
                            pdbs: Optional[list] = None):
        """cluster.go:145-184: exactly one of (NodeToBeRemoved, UnremovableNode) is set."""
        from .planner import RemainingPdbTracker
        tracker = RemainingPdbTracker()
        tracker.SetPdbs(pdbs or [])
        if self.can_persist:
            rem, unrem = self.SimulateNodeRemovals([node_name], destination_map, timestamp, tracker)
        else:
            rem, unrem = self.FindNodesToRemove([node_name], list(destination_map), timestamp, tracker.GetPdbs())
        return (rem[0] if rem else None), (unrem[0] if unrem else None)

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
