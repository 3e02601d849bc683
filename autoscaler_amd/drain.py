"""Host-side drain policy: which pods of a node must move (CA/utils/drain, CA/simulator/drain.go).

GetPodsToMove / GetPodsForDeletionOnNodeDrain classify pods with listers,
annotations and PDBs; they need API objects, so they stay on the host and the
device receives only the verdict.  This is the subset of
drain.go:76-232 the simulation needs: mirror pods, long-terminating pods,
DaemonSet / replicated / unreplicated pods, kube-system, local storage, the
safe-to-evict annotations, and the PDB check of simulator/drain.go:73-90.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

from .k8s import Pod, is_daemonset_pod

PodSafeToEvictKey = "cluster-autoscaler.kubernetes.io/safe-to-evict"       # drain.go:42
ConfigMirrorAnnotationKey = "kubernetes.io/config.mirror"
PodLongTerminatingExtraThreshold = 30.0                                    # drain.go:34
DefaultTerminationGracePeriodSeconds = 30                                  # core/v1 types.go

# BlockingPodReason (drain.go:51-73)
NoReason, ControllerNotFound, MinReplicasReached, NotReplicated, LocalStorageRequested, \
    NotSafeToEvictAnnotation, UnmovableKubeSystemPod, NotEnoughPdb, UnexpectedError = range(9)


@dataclass
class BlockingPod:
    pod: Pod
    reason: int


@dataclass
class NodeDeleteOptions:
    """simulator.NodeDeleteOptions (CA/simulator/drain.go:33-41)."""
    skip_nodes_with_system_pods: bool = True
    skip_nodes_with_local_storage: bool = True
    min_replica_count: int = 0


@dataclass
class ListerRegistry:
    """Existence/replica counts of controllers: kind -> {(namespace, name): replicas or None}."""
    objects: dict = field(default_factory=dict)

    def get(self, kind: str, namespace: str, name: str):
        return self.objects.get(kind, {}).get((namespace, name), "missing")


@dataclass
class PodDisruptionBudget:
    namespace: str
    match_labels: dict
    disruptions_allowed: int


def is_mirror_pod(p: Pod) -> bool:
    return ConfigMirrorAnnotationKey in p.annotations


def has_local_storage(p: Pod) -> bool:
    """HasLocalStorage / isLocalVolume (drain.go:253-265)."""
    return any(v in ("emptyDir", "hostPath") for v in p.volumes)


def is_pod_long_terminating(p: Pod, now: float) -> bool:
    """IsPodLongTerminating (drain.go:293-306): DeletionTimestamp + grace (nil -> 30 s) +
    PodLongTerminatingExtraThreshold is strictly before now."""
    if p.deletion_timestamp is None:
        return False
    grace = p.termination_grace_period_seconds
    if grace is None:
        grace = DefaultTerminationGracePeriodSeconds
    return p.deletion_timestamp + grace + PodLongTerminatingExtraThreshold < now


def is_pod_terminal(p: Pod) -> bool:
    """isPodTerminal (drain.go:239-251)."""
    if p.restart_policy == "Never" and p.phase in ("Succeeded", "Failed"):
        return True
    if p.restart_policy == "OnFailure" and p.phase == "Succeeded":
        return True
    return p.phase == "Failed"


def get_pods_for_deletion_on_node_drain(pods: list, pdbs: list, skip_system: bool, skip_local: bool,
                                        listers: Optional[ListerRegistry], min_replica: int, now: float = 0.0):
    """drain.GetPodsForDeletionOnNodeDrain (drain.go:76-232)."""
    out, ds = [], []
    check_refs = listers is not None
    ks_pdbs = [p for p in pdbs if p.namespace == "kube-system"]
    for pod in pods:
        if is_mirror_pod(pod):
            continue
        if is_pod_long_terminating(pod, now):                                  # :107-112
            continue
        is_ds = False
        replicated = False
        safe = pod.annotations.get(PodSafeToEvictKey) == "true"
        terminal = is_pod_terminal(pod)
        ref = pod.controller_ref()
        kind = ref.kind if ref else ""
        # branch order of drain.go:129-205: ReplicationController, IsDaemonSetPod, Job,
        # ReplicaSet, StatefulSet
        if kind == "ReplicationController":
            if check_refs:
                obj = listers.get(kind, pod.namespace, ref.name)
                if obj == "missing":
                    return [], [], BlockingPod(pod, ControllerNotFound), "controller not found"
                if obj is not None and obj < min_replica:
                    return [], [], BlockingPod(pod, MinReplicasReached), "too few replicas"
            replicated = True
        elif is_daemonset_pod(pod):
            is_ds = True
            if check_refs and kind == "DaemonSet" and listers.get("DaemonSet", pod.namespace, ref.name) == "missing":
                return [], [], BlockingPod(pod, ControllerNotFound), "daemonset not found"
        elif kind == "ReplicaSet":
            if check_refs:
                obj = listers.get(kind, pod.namespace, ref.name)
                if obj == "missing":
                    return [], [], BlockingPod(pod, ControllerNotFound), "controller not found"
                if obj is not None and obj < min_replica:
                    return [], [], BlockingPod(pod, MinReplicasReached), "too few replicas"
            replicated = True
        elif kind in ("Job", "StatefulSet"):
            if check_refs and listers.get(kind, pod.namespace, ref.name) == "missing":
                return [], [], BlockingPod(pod, ControllerNotFound), f"{kind} not found"
            replicated = True
        if is_ds:
            ds.append(pod)
            continue
        if not safe and not terminal:
            if not replicated:
                return [], [], BlockingPod(pod, NotReplicated), f"{pod.namespace}/{pod.name} is not replicated"
            if pod.namespace == "kube-system" and skip_system:
                if not any(all(pod.labels.get(k) == v for k, v in b.match_labels.items()) for b in ks_pdbs):
                    return [], [], BlockingPod(pod, UnmovableKubeSystemPod), "kube-system pod"
            if has_local_storage(pod) and skip_local:
                return [], [], BlockingPod(pod, LocalStorageRequested), "local storage"
            if pod.annotations.get(PodSafeToEvictKey) == "false":
                return [], [], BlockingPod(pod, NotSafeToEvictAnnotation), "not safe to evict"
        out.append(pod)
    return out, ds, None, None


def pdb_matches(pdb: "PodDisruptionBudget", pod: Pod) -> bool:
    """Namespace + selector match of checkPdbs / RemainingPdbTracker (drain.go:82, basic.go:71)."""
    return pod.namespace == pdb.namespace and all(pod.labels.get(k) == v for k, v in pdb.match_labels.items())


def get_pods_to_move(node_pods: list, options: NodeDeleteOptions, listers: Optional[ListerRegistry],
                     pdbs: list, now: float = 0.0, check_pdbs: bool = True):
    """simulator.GetPodsToMove (CA/simulator/drain.go:50-90).  check_pdbs=False leaves out the
    budget check (:64-66), for callers that apply it against changing budgets themselves."""
    pods, ds, blocking, err = get_pods_for_deletion_on_node_drain(
        node_pods, pdbs, options.skip_nodes_with_system_pods, options.skip_nodes_with_local_storage, listers,
        options.min_replica_count, now)
    if err is not None or not check_pdbs:
        return pods, ds, blocking, err
    for pdb in pdbs:                                   # checkPdbs (:73-90)
        for pod in pods:
            if pod.namespace == pdb.namespace and all(pod.labels.get(k) == v for k, v in pdb.match_labels.items()):
                if pdb.disruptions_allowed < 1:
                    return [], [], BlockingPod(pod, NotEnoughPdb), "not enough pod disruption budget"
    return pods, ds, None, None
