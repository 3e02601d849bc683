"""Kernel scope classifier.

The kernels implement the six default-profile filter plugins of the path
(NodeUnschedulable, NodeName, TaintToleration, NodeAffinity, NodePorts,
NodeResourcesFit).  The other default filters are no-ops for a pod without the
features they read; a pod WITH them, or any simulation while the snapshot holds a
pod with required anti-affinity, must run on the reference (Go) path.  The
classification is conservative: a feature that MAY make a plugin act is enough.

  InterPodAffinity  PreFilter Skips only when the pod has no required pod
                    (anti-)affinity terms and no existing pod's required
                    anti-affinity matches it (vendored
                    SF/plugins/interpodaffinity/filtering.go:230-268; existing
                    anti-affinity counted from HavePodsWithRequiredAntiAffinityList).
  PodTopologySpread Filter is a no-op without DoNotSchedule constraints: only
                    DoNotSchedule constraints are kept (podtopologyspread/
                    filtering.go:238-258), and the system defaults are ScheduleAnyway.
  Volume plugins    VolumeBinding / VolumeZone Skip without PVC or ephemeral
                    volumes (volumebinding/volume_binding.go:112-169,
                    volumezone/volume_zone.go:97-103); VolumeRestrictions acts on
                    GCE PD / AWS EBS / RBD / iSCSI and ReadWriteOncePod PVCs
                    (volumerestrictions/volume_restrictions.go:166-176, :133-149);
                    NodeVolumeLimits counts PVC, ephemeral and migratable in-tree
                    volumes (nodevolumelimits/csi.go:150-175, non_csi.go:212-330).
                    Only the volume kinds below are read by none of them.
"""
from __future__ import annotations

from typing import Optional

from .k8s import Pod

# volume sources no volume filter plugin reads (every other kind is out of scope)
IN_SCOPE_VOLUMES = frozenset({"emptyDir", "hostPath", "configMap", "secret", "downwardAPI", "projected",
                              "gitRepo", "nfs"})


class UnsupportedByKernels(RuntimeError):
    """CA_EUNSUPPORTED: the caller must use the reference (Go) path for this input."""


def _when_unsatisfiable(c) -> str:
    if isinstance(c, dict):
        return c.get("whenUnsatisfiable", c.get("when_unsatisfiable", ""))
    return getattr(c, "when_unsatisfiable", "")


def has_required_anti_affinity(pod: Pod) -> bool:
    a = pod.affinity
    return a is not None and bool(a.required_anti_affinity)


def out_of_scope_reason(pod: Pod) -> Optional[str]:
    """Why `pod` needs a plugin the kernels do not implement, or None."""
    a = pod.affinity
    if a is not None and (a.required_pod_affinity or a.required_anti_affinity):
        return "InterPodAffinity: required pod (anti-)affinity terms"
    if any(_when_unsatisfiable(c) == "DoNotSchedule" for c in pod.topology_spread):
        return "PodTopologySpread: DoNotSchedule constraint"
    for v in pod.volumes:
        if v not in IN_SCOPE_VOLUMES:
            return f"volume plugins: {v} volume"
    return None
