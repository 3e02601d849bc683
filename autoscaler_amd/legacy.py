"""Legacy scale-down bookkeeping around the removal sweep (CA/core/scaledown/legacy).

``ScaleDown.UpdateUnneededNodes`` (legacy.go:101-225) is the caller of the sweep in
every RunOnce (static_autoscaler.go:615 -> wrapper.go:50-52): per-node eligibility and
utilization (eligibility.go:66-176), the empty nodes (legacy.go:358-422 over
FindEmptyNodesToRemove), the candidate split (chooseCandidates :468-484),
FindNodesToRemove over the candidates and an additional pool (:146-176), and the
unneeded / unremovable node books (unneeded.go, unremovable/nodes.go:50-112).  The
policy parts are host code (O(nodes) bookkeeping); both sweeps and the
utilization pass run on the device through the facades.  Used to pin the path against
the reference's TestFindUnneededNodes (legacy_test.go:58-216).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Optional

from . import simulator as sim
from . import utilization
from .clustersnapshot import ClusterSnapshot
from .k8s import Node

ScaleDownDisabledKey = "cluster-autoscaler.kubernetes.io/scale-down-disabled"   # eligibility.go:38
ToBeDeletedTaint = "ToBeDeletedByClusterAutoscaler"                             # utils/taints/taints.go:38
MaxKubernetesEmptyNodeDeletionTime = 3 * 60.0                                    # delete_in_batch.go:42
MaxCloudProviderNodeDeletionTime = 5 * 60.0                                      # delete_in_batch.go:44


@dataclass
class NodeGroup:
    """The cloudprovider.NodeGroup fields scale-down reads."""
    id: str
    min_size: int
    max_size: int
    target_size: int


@dataclass
class ScaleDownOptions:
    """The config.AutoscalingOptions fields UpdateUnneededNodes reads."""
    scale_down_utilization_threshold: float = 0.5
    scale_down_gpu_utilization_threshold: float = 0.5
    unremovable_node_recheck_timeout: float = 5 * 60.0
    scale_down_non_empty_candidates_count: int = 30
    scale_down_candidates_pool_ratio: float = 0.1
    scale_down_candidates_pool_min_count: int = 50
    scale_down_unready_enabled: bool = False
    ignore_daemonsets_utilization: bool = False
    ignore_mirror_pods_utilization: bool = False


def to_be_deleted_time(node: Node) -> Optional[float]:
    """taints.GetToBeDeletedTime (taints.go:180-202): the taint value as unix seconds."""
    for t in node.taints:
        if t.key == ToBeDeletedTaint:
            try:
                return float(int(t.value))
            except ValueError:
                return None
    return None


def is_node_being_deleted(node: Node, timestamp: float) -> bool:
    """actuation.IsNodeBeingDeleted (delete_in_batch.go:179-182)."""
    t = to_be_deleted_time(node)
    return t is not None and (timestamp - t < MaxCloudProviderNodeDeletionTime
                              or timestamp - t < MaxKubernetesEmptyNodeDeletionTime)


class UnremovableNodes:
    """unremovable.Nodes (unremovable/nodes.go:30-112): reasons of this loop, TTLs across loops."""

    def __init__(self):
        self.reasons: dict = {}
        self.ttls: dict = {}

    def Update(self, snapshot: ClusterSnapshot, timestamp: float) -> None:  # noqa: N802
        self.reasons = {}
        names = set(snapshot.node_names())
        self.ttls = {n: ttl for n, ttl in self.ttls.items() if n in names and ttl > timestamp}

    def Add(self, u: sim.UnremovableNode) -> None:  # noqa: N802
        self.reasons[u.node.name] = u

    def AddTimeout(self, u: sim.UnremovableNode, timeout: float) -> None:  # noqa: N802
        self.ttls[u.node.name] = timeout
        self.Add(u)

    def AddReason(self, node: Node, reason: int) -> None:  # noqa: N802
        self.Add(sim.UnremovableNode(node, reason))

    def AsList(self) -> list:  # noqa: N802
        return list(self.reasons.values())

    def HasReason(self, name: str) -> bool:  # noqa: N802
        return name in self.reasons

    def IsRecent(self, name: str) -> bool:  # noqa: N802
        return name in self.ttls


class UnneededNodes:
    """unneeded.Nodes (core/scaledown/unneeded/nodes.go): the current set with since-times."""

    def __init__(self):
        self.since: dict = {}

    def Update(self, to_remove: list, timestamp: float) -> None:  # noqa: N802
        self.since = {t.node.name: self.since.get(t.node.name, timestamp) for t in to_remove}

    def Contains(self, name: str) -> bool:  # noqa: N802
        return name in self.since

    def AsList(self) -> list:  # noqa: N802
        return list(self.since)


class ScaleDown:
    """legacy.ScaleDown (legacy.go:56-99) restricted to UpdateUnneededNodes."""

    def __init__(self, snapshot: ClusterSnapshot, removal_simulator: sim.RemovalSimulator, node_groups: dict,
                 options: ScaleDownOptions, gpu_configs: Optional[dict] = None,
                 calculate_all: Optional[Callable] = None):
        self.snapshot = snapshot
        self.removal_simulator = removal_simulator
        self.node_groups = node_groups                 # node name -> NodeGroup (NodeGroupForNode)
        self.options = options
        self.gpu_configs = gpu_configs or {}           # node name -> utilization.GpuConfig
        self.calculate_all = calculate_all or utilization.CalculateAll
        self.unneeded_nodes = UnneededNodes()
        self.unremovable_nodes = UnremovableNodes()
        self.node_utilization_map: dict = {}

    # eligibility.FilterOutUnremovable (eligibility.go:66-103)
    def _filter_out_unremovable(self, candidates: list, timestamp: float):
        ineligible, util_map, unneeded = [], {}, []
        names = set(self.snapshot.node_names())
        resolved = [n for n in candidates if n.name in names]
        infos = {n.name: self.snapshot.Get(n.name) for n in resolved}
        todo = [n for n in resolved if not self.unremovable_nodes.IsRecent(n.name)
                and not is_node_being_deleted(n, timestamp) and n.annotations.get(ScaleDownDisabledKey) != "true"]
        calc = dict(zip([n.name for n in todo],
                        self.calculate_all([infos[n.name] for n in todo], self.options.ignore_daemonsets_utilization,
                                           self.options.ignore_mirror_pods_utilization,
                                           [self.gpu_configs.get(n.name) for n in todo], timestamp))) if todo else {}
        for node in candidates:
            if node.name not in names:
                ineligible.append(sim.UnremovableNode(node, sim.UnexpectedError))
                continue
            if self.unremovable_nodes.IsRecent(node.name):
                ineligible.append(sim.UnremovableNode(node, sim.RecentlyUnremovable))
                continue
            reason, info = self._reason_and_utilization(node, calc.get(node.name), timestamp)
            if info is not None:
                util_map[node.name] = info
            if reason != sim.NoReason:
                ineligible.append(sim.UnremovableNode(node, reason))
                continue
            unneeded.append(node.name)
        return unneeded, util_map, ineligible

    # unremovableReasonAndNodeUtilization (eligibility.go:105-156)
    def _reason_and_utilization(self, node: Node, calc, timestamp: float):
        if is_node_being_deleted(node, timestamp):
            return sim.CurrentlyBeingDeleted, None
        if node.annotations.get(ScaleDownDisabledKey) == "true":
            return sim.ScaleDownDisabledAnnotation, None
        info, _err = calc                                  # an error only logs (:125-128)
        ng = self.node_groups.get(node.name)
        if ng is None:
            return sim.NotAutoscaled, None
        if not self.options.scale_down_unready_enabled and not node.ready:
            return sim.ScaleDownUnreadyDisabled, None
        gpu = self.gpu_configs.get(node.name) is not None
        threshold = (self.options.scale_down_gpu_utilization_threshold if gpu
                     else self.options.scale_down_utilization_threshold)
        if info.Utilization >= threshold:                  # isNodeBelowUtilizationThreshold (:158-178)
            return sim.NotUnderutilized, info
        return sim.NoReason, info

    # getEmptyNodesToRemove (legacy.go:364-422) without resource limits
    def _empty_nodes_to_remove(self, candidates: list, timestamp: float) -> list:
        empty = self.removal_simulator.FindEmptyNodesToRemove(candidates, timestamp)
        available: dict = {}
        out = []
        for name in empty:
            ng = self.node_groups.get(name)
            if ng is None:
                continue
            if ng.id not in available:
                available[ng.id] = max(ng.target_size - ng.min_size, 0)
            if available[ng.id] > 0:
                available[ng.id] -= 1
                out.append(sim.NodeToBeRemoved(self.snapshot.Get(name).node, []))
        return out

    def _choose_candidates(self, nodes: list):
        """chooseCandidates (legacy.go:468-484)."""
        if self.options.scale_down_non_empty_candidates_count <= 0:
            return nodes, []
        cand = [n for n in nodes if self.unneeded_nodes.Contains(n)]
        non = [n for n in nodes if not self.unneeded_nodes.Contains(n)]
        return cand, non

    def UpdateUnneededNodes(self, destination_nodes: list, scale_down_candidates: list,  # noqa: N802
                            timestamp: float) -> None:
        """legacy.go:101-225."""
        all_nodes = self.snapshot.node_names()
        self.unremovable_nodes.Update(self.snapshot, timestamp)
        unneeded, util_map, ineligible = self._filter_out_unremovable(scale_down_candidates, timestamp)
        for u in ineligible:
            self.unremovable_nodes.Add(u)
        empty = self._empty_nodes_to_remove(unneeded, timestamp)
        empty_names = {e.node.name for e in empty}
        non_empty = [n for n in unneeded if n not in empty_names]
        cand, non = self._choose_candidates(non_empty)
        dest = [n.name for n in destination_nodes]
        to_remove, unremovable = self.removal_simulator.FindNodesToRemove(cand, dest, timestamp, [])
        extra = self.options.scale_down_non_empty_candidates_count - len(to_remove)
        extra = min(extra, len(non))
        pool = int(math.ceil(len(all_nodes) * self.options.scale_down_candidates_pool_ratio))
        pool = min(max(pool, self.options.scale_down_candidates_pool_min_count), len(non))
        if extra > 0:
            more, more_un = self.removal_simulator.FindNodesToRemove(non[:pool], dest, timestamp, [])
            to_remove += more[:extra]
            unremovable += more_un
        to_remove += empty
        self.unneeded_nodes.Update(to_remove, timestamp)
        if unremovable:
            timeout = timestamp + self.options.unremovable_node_recheck_timeout
            for u in unremovable:
                self.unremovable_nodes.AddTimeout(u, timeout)
        for node in scale_down_candidates:
            if not self.unneeded_nodes.Contains(node.name) and not self.unremovable_nodes.HasReason(node.name):
                self.unremovable_nodes.AddReason(node, sim.NotUnneededOtherReason)
        self.removal_simulator.DropOldHints()
        self.node_utilization_map = util_map
