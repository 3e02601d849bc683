"""Minimal Kubernetes API objects used by the host side of the boundary.

Only the fields the scheduling-simulation path reads are modelled (k8s.io/api
v0.27 core/v1 names, snake_cased).  Quantities follow
k8s.io/apimachinery/pkg/api/resource: values are exact decimals, ``MilliValue``
and ``Value`` round up (quantity.go:743-764).

Builders mirror CA/utils/test/test_utils.go (BuildTestPod :36-68, BuildTestNode
:179-210, AddGpusToNode :221-233, ...), so tests read like the reference's tests.
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field
from fractions import Fraction
from typing import Optional

# ---------------------------------------------------------------------------
# quantities
# ---------------------------------------------------------------------------
_SUFFIX = {
    "": Fraction(1), "m": Fraction(1, 1000), "k": Fraction(1000), "M": Fraction(10 ** 6), "G": Fraction(10 ** 9),
    "T": Fraction(10 ** 12), "P": Fraction(10 ** 15), "E": Fraction(10 ** 18), "n": Fraction(1, 10 ** 9),
    "u": Fraction(1, 10 ** 6), "Ki": Fraction(1024), "Mi": Fraction(1024 ** 2), "Gi": Fraction(1024 ** 3),
    "Ti": Fraction(1024 ** 4), "Pi": Fraction(1024 ** 5), "Ei": Fraction(1024 ** 6),
}
_QRE = re.compile(r"^([+-]?[0-9.]+)([eE][+-]?[0-9]+)?(Ki|Mi|Gi|Ti|Pi|Ei|m|k|M|G|T|P|E|n|u)?$")


class Quantity:
    """An exact resource quantity (resource.Quantity)."""

    __slots__ = ("v",)

    def __init__(self, v):
        if isinstance(v, Quantity):
            self.v = v.v
        elif isinstance(v, str):
            m = _QRE.match(v.strip())
            if not m:
                raise ValueError(f"bad quantity {v!r}")
            num = Fraction(m.group(1))
            if m.group(2):
                num *= Fraction(10) ** int(m.group(2)[1:])
            self.v = num * _SUFFIX[m.group(3) or ""]
        else:
            self.v = Fraction(v)

    @staticmethod
    def milli(m: int) -> "Quantity":
        """resource.NewMilliQuantity"""
        return Quantity(Fraction(m, 1000))

    def milli_value(self) -> int:   # quantity.go:749 MilliValue: ceil(v*1000)
        return math.ceil(self.v * 1000)

    def value(self) -> int:          # quantity.go:743 Value: ceil(v)
        return math.ceil(self.v)

    def __add__(self, o: "Quantity") -> "Quantity":
        return Quantity(self.v + Quantity(o).v)

    def __repr__(self) -> str:
        return f"Quantity({self.v})"


def cpu(milli: int) -> Quantity:
    return Quantity.milli(milli)


# ---------------------------------------------------------------------------
# objects
# ---------------------------------------------------------------------------
@dataclass
class ContainerPort:
    host_port: int = 0
    host_ip: str = ""
    protocol: str = ""
    container_port: int = 0


@dataclass
class Container:
    requests: dict = field(default_factory=dict)      # resource name -> Quantity
    ports: list = field(default_factory=list)


@dataclass
class Toleration:
    key: str = ""
    operator: str = ""          # "" == Equal
    value: str = ""
    effect: str = ""


@dataclass
class Taint:
    key: str
    value: str = ""
    effect: str = "NoSchedule"


@dataclass
class NodeSelectorRequirement:
    key: str
    operator: str               # In NotIn Exists DoesNotExist Gt Lt
    values: list = field(default_factory=list)


@dataclass
class NodeSelectorTerm:
    match_expressions: list = field(default_factory=list)
    match_fields: list = field(default_factory=list)


@dataclass
class Affinity:
    # nil vs present matters: None == RequiredDuringSchedulingIgnoredDuringExecution nil
    required_terms: Optional[list] = None
    pod_affinity: bool = False            # any PodAffinity / PodAntiAffinity present
    required_anti_affinity: bool = False  # PodAntiAffinity.RequiredDuringScheduling... terms present
    required_pod_affinity: bool = False   # PodAffinity.RequiredDuringScheduling... terms present


@dataclass
class TopologySpreadConstraint:
    """v1.TopologySpreadConstraint (the fields the scope classifier reads)."""
    max_skew: int = 1
    topology_key: str = ""
    when_unsatisfiable: str = "DoNotSchedule"     # DoNotSchedule | ScheduleAnyway
    match_labels: dict = field(default_factory=dict)


@dataclass
class OwnerReference:
    kind: str
    name: str
    uid: str = ""
    controller: bool = True


@dataclass
class Pod:
    name: str
    namespace: str = "default"
    uid: str = ""
    labels: dict = field(default_factory=dict)
    annotations: dict = field(default_factory=dict)
    containers: list = field(default_factory=list)
    init_containers: list = field(default_factory=list)
    overhead: Optional[dict] = None
    node_name: str = ""
    node_selector: Optional[dict] = None
    affinity: Optional[Affinity] = None
    tolerations: list = field(default_factory=list)
    owner_refs: list = field(default_factory=list)
    volumes: list = field(default_factory=list)
    topology_spread: list = field(default_factory=list)
    phase: str = "Running"
    deletion_timestamp: Optional[float] = None
    priority: Optional[int] = None                  # Spec.Priority (corev1helpers.PodPriority: nil -> 0)
    termination_grace_period_seconds: Optional[int] = None   # Spec.TerminationGracePeriodSeconds
    restart_policy: str = "Always"                  # Spec.RestartPolicy (Always | OnFailure | Never)

    def controller_ref(self) -> Optional[OwnerReference]:
        for r in self.owner_refs:
            if r.controller:
                return r
        return None

    def key(self) -> str:
        return f"{self.namespace}/{self.name}"


@dataclass
class Node:
    name: str
    labels: dict = field(default_factory=dict)
    taints: list = field(default_factory=list)
    allocatable: dict = field(default_factory=dict)    # resource name -> Quantity
    unschedulable: bool = False
    annotations: dict = field(default_factory=dict)
    ready: bool = True                                 # NodeReady condition (kube_util.GetReadinessState)


# ---------------------------------------------------------------------------
# builders (CA/utils/test/test_utils.go)
# ---------------------------------------------------------------------------
def build_test_pod(name: str, cpu_milli: int, mem: int) -> Pod:
    """BuildTestPod (test_utils.go:36-68): UID = name, namespace default, one container."""
    req = {}
    if cpu_milli >= 0:
        req["cpu"] = Quantity.milli(cpu_milli)
    if mem >= 0:
        req["memory"] = Quantity(mem)
    return Pod(name=name, uid=name, containers=[Container(requests=req)])


def build_scheduled_test_pod(name: str, cpu_milli: int, mem: int, node_name: str) -> Pod:
    p = build_test_pod(name, cpu_milli, mem)
    p.node_name = node_name
    return p


def build_test_node(name: str, millicpu: int, mem: int, pods: int = 100) -> Node:
    """BuildTestNode (test_utils.go:179-210): capacity == allocatable, pods = 100."""
    alloc = {"pods": Quantity(pods)}
    if millicpu >= 0:
        alloc["cpu"] = Quantity.milli(millicpu)
    if mem >= 0:
        alloc["memory"] = Quantity(mem)
    return Node(name=name, allocatable=alloc)


def add_gpus_to_node(node: Node, count: int) -> None:
    """AddGpusToNode (test_utils.go:221-233)."""
    node.taints.append(Taint("nvidia.com/gpu", "present", "NoSchedule"))
    node.allocatable["nvidia.com/gpu"] = Quantity(count)
    node.labels["cloud.google.com/gke-accelerator"] = "nvidia-tesla-k80"


def request_gpu_for_pod(pod: Pod, count: int) -> None:
    """RequestGpuForPod (test_utils.go:161-172)."""
    pod.containers[0].requests["nvidia.com/gpu"] = Quantity(count)


def tolerate_gpu_for_pod(pod: Pod) -> None:
    """TolerateGpuForPod (test_utils.go:175-177)."""
    pod.tolerations.append(Toleration(key="nvidia.com/gpu", operator="Exists"))


def set_rs_pod(pod: Pod, rs_name: str) -> Pod:
    pod.owner_refs = [OwnerReference("ReplicaSet", rs_name, rs_name)]
    return pod


def set_ds_pod(pod: Pod) -> Pod:
    pod.owner_refs = [OwnerReference("DaemonSet", "ds", "api/v1/namespaces/default/daemonsets/ds")]
    return pod


DAEMONSET_POD_ANNOTATION = "cluster-autoscaler.kubernetes.io/daemonset-pod"   # utils/pod/pod.go:26-27


def is_daemonset_pod(pod: Pod) -> bool:
    """pod_util.IsDaemonSetPod (CA/utils/pod/pod.go:32-43): controller kind DaemonSet, or the
    cluster-autoscaler.kubernetes.io/daemonset-pod=true annotation."""
    ref = pod.controller_ref()
    if ref is not None and ref.kind == "DaemonSet":
        return True
    return pod.annotations.get(DAEMONSET_POD_ANNOTATION) == "true"


def set_mirror_pod(pod: Pod) -> Pod:
    pod.annotations["kubernetes.io/config.mirror"] = "mirror"
    return pod
