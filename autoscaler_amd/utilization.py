"""Scale-down eligibility: ``utilization.Calculate`` and ``FindEmptyNodesToRemove`` over
every node in one HIP launch.

Mirrors ``CA/simulator/utilization/info.go:34-127`` (``Info``, ``Calculate``,
``calculateUtilizationOfResource``) and ``RemovalSimulator.FindEmptyNodesToRemove``
(``CA/simulator/cluster.go:187-202``).  The host turns each NodeInfo into one
``ca_util_node`` row and its pods into ``ca_util_pod`` rows (request MilliValues, the
DaemonSet / mirror / deleted flags, and the per-pod ``GetPodsToMove`` verdict with nil
listers, which stays on the host: SURVEY.md §8a A18); ``libcasim.so`` does the per-node
reductions and the float64 ratios.  There is no CPU fallback: without the HIP library
every entry point raises.

Requests are summed as per-pod MilliValues where the reference sums Quantities and takes
one MilliValue (info.go:122-126); the two agree whenever each request is a whole number of
milli-units (cpu in m, memory in bytes, GPU counts).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import abi
from .drain import get_pods_for_deletion_on_node_drain, is_mirror_pod
from .k8s import Node, Pod, is_daemonset_pod

ResourceCPU, ResourceMemory = "cpu", "memory"
DaemonSetPodAnnotationKey = "cluster-autoscaler.kubernetes.io/daemonset-pod"   # utils/pod/pod.go:27
DefaultTerminationGracePeriodSeconds = 30                                      # core/v1/types.go

_RESOURCE_NAME = {abi.CA_UTIL_CPU: ResourceCPU, abi.CA_UTIL_MEM: ResourceMemory}
_ERRORS = {
    abi.CA_UTIL_NO_CPU: "failed to get cpu from {}", abi.CA_UTIL_ZERO_CPU: "cpu is 0 at {}",
    abi.CA_UTIL_NO_MEM: "failed to get memory from {}", abi.CA_UTIL_ZERO_MEM: "memory is 0 at {}",
}


@dataclass
class GpuConfig:
    """cloudprovider.GpuConfig (CA/cloudprovider/cloud_provider.go)."""
    label: str
    type: str
    resource_name: str


@dataclass
class Info:
    """utilization.Info (info.go:34-43)."""
    CpuUtil: float = 0.0
    MemUtil: float = 0.0
    GpuUtil: float = 0.0
    ResourceName: str = ""
    Utilization: float = 0.0


class UtilizationError(Exception):
    pass




def _milli(reqs: list, name: str) -> int:
    return sum(c.requests[name].milli_value() for c in reqs if name in c.requests)


def node_row(node: Node, gpu_config: Optional[GpuConfig]) -> np.ndarray:
    row = np.zeros((), abi.UTIL_NODE_DTYPE)
    flags = 0
    for i, (name, bit) in enumerate(((ResourceCPU, abi.CA_UNODE_HAS_CPU), (ResourceMemory, abi.CA_UNODE_HAS_MEM))):
        if name in node.allocatable:
            flags |= bit
            row["alloc_milli"][i] = node.allocatable[name].milli_value()
    if gpu_config is not None:
        flags |= abi.CA_UNODE_GPU_CONFIG
        if gpu_config.resource_name in node.allocatable:
            flags |= abi.CA_UNODE_HAS_GPU
            row["alloc_milli"][2] = node.allocatable[gpu_config.resource_name].milli_value()
    row["flags"] = flags
    return row


def pod_row(p: Pod, gpu_resource: Optional[str]) -> np.ndarray:
    row = np.zeros((), abi.UTIL_POD_DTYPE)
    row["req_milli"][0] = _milli(p.containers, ResourceCPU)          # containers only (info.go:102,122)
    row["req_milli"][1] = _milli(p.containers, ResourceMemory)
    if gpu_resource:
        row["req_milli"][2] = _milli(p.containers, gpu_resource)
    flags = 0
    if is_daemonset_pod(p):
        flags |= abi.CA_UPOD_DAEMONSET
    if is_mirror_pod(p):
        flags |= abi.CA_UPOD_MIRROR
    if p.deletion_timestamp is not None:
        flags |= abi.CA_UPOD_DELETED
        row["deletion_ns"] = round(p.deletion_timestamp * 1e9)
        g = p.termination_grace_period_seconds
        row["grace_s"] = DefaultTerminationGracePeriodSeconds if g is None else g
    row["flags"] = flags
    return row


def drain_flags(p: Pod, delete_options, now: float) -> int:
    """The pod's share of GetPodsToMove(nodeInfo, deleteOptions, nil, nil, ts)
    (CA/simulator/drain.go:50-90): with nil listers and no PDBs each pod is classified on
    its own, so a node's call fails iff one of its pods blocks and lists the movable ones."""
    pods, _, _, err = get_pods_for_deletion_on_node_drain(
        [p], [], delete_options.skip_nodes_with_system_pods, delete_options.skip_nodes_with_local_storage, None,
        delete_options.min_replica_count, now)
    if err is not None:
        return abi.CA_UPOD_BLOCKING
    return abi.CA_UPOD_MOVABLE if pods else 0


def build_table(node_infos: list, gpu_configs: list, delete_options=None, now: float = 0.0):
    """Rows for ca_util_table_create: (nodes, pod_off, pods)."""
    nodes = np.zeros(len(node_infos), abi.UTIL_NODE_DTYPE)
    pod_off = np.zeros(len(node_infos) + 1, np.int32)
    rows = []
    for i, (ni, gc) in enumerate(zip(node_infos, gpu_configs)):
        nodes[i] = node_row(ni.node, gc)
        for p in ni.pods:
            r = pod_row(p, gc.resource_name if gc else None)
            if delete_options is not None:
                r["flags"] |= drain_flags(p, delete_options, now)
            rows.append(r)
        pod_off[i + 1] = len(rows)
    pods = np.array(rows, abi.UTIL_POD_DTYPE) if rows else np.zeros(0, abi.UTIL_POD_DTYPE)
    return nodes, pod_off, pods


def info_from_row(r, node_name: str, gpu_config: Optional[GpuConfig]):
    """(Info, error) of one ca_util_info row, as Calculate returns them."""
    st = int(r["status"])
    if st != abi.CA_UTIL_OK:
        return Info(), UtilizationError(_ERRORS[st].format(node_name))
    res = int(r["resource"])
    name = gpu_config.resource_name if res == abi.CA_UTIL_GPU else _RESOURCE_NAME[res]
    return Info(float(r["cpu"]), float(r["mem"]), float(r["gpu"]), name, float(r["utilization"])), None


def CalculateAll(node_infos: list, skip_daemonset_pods: bool, skip_mirror_pods: bool,  # noqa: N802
                 gpu_configs: Optional[list], current_time: float, device: int = 0):
    """Calculate for every NodeInfo in one launch; returns [(Info, error)] in input order."""
    from .native import UtilTable
    gpu_configs = gpu_configs if gpu_configs is not None else [None] * len(node_infos)
    nodes, pod_off, pods = build_table(node_infos, gpu_configs)
    t = UtilTable(device, nodes, pod_off, pods)
    try:
        out = t.calculate(skip_daemonset_pods, skip_mirror_pods, round(current_time * 1e9))
    finally:
        t.close()
    return [info_from_row(out[i], ni.node.name, gc) for i, (ni, gc) in enumerate(zip(node_infos, gpu_configs))]


def Calculate(node_info, skip_daemonset_pods: bool, skip_mirror_pods: bool,  # noqa: N802
              gpu_config: Optional[GpuConfig], current_time: float):
    """utilization.Calculate (info.go:48-81) for one node: returns (Info, error)."""
    return CalculateAll([node_info], skip_daemonset_pods, skip_mirror_pods, [gpu_config], current_time)[0]


def FindEmptyNodesToRemove(node_infos: list, delete_options, timestamp: float = 0.0,  # noqa: N802
                           device: int = 0) -> list:
    """RemovalSimulator.FindEmptyNodesToRemove (cluster.go:187-202) over resolved NodeInfos
    (candidates missing from the snapshot are dropped by the caller, :191-194)."""
    from .native import UtilTable
    nodes, pod_off, pods = build_table(node_infos, [None] * len(node_infos), delete_options, timestamp)
    t = UtilTable(device, nodes, pod_off, pods)
    try:
        out = t.calculate(False, False, round(timestamp * 1e9))
    finally:
        t.close()
    return [ni.node.name for i, ni in enumerate(node_infos) if out[i]["empty"]]
