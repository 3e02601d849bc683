"""BinpackingNodeEstimator over the mirror (CA/estimator).

Estimator.Estimate(pods, nodeTemplate, nodeGroup) -> (node count, scheduled pods)
with the reference's semantics (binpacking_estimator.go:65-193) and the
thresholdBasedEstimationLimiter (threshold_based_limiter.go:27-64).  The limiter's
wall-clock cap is non-deterministic in the reference; only the
node cap is implemented, a non-zero duration raises.

``estimate_batch`` runs the Estimate of several node groups in one device call,
sharing the checker's lastIndex exactly as consecutive Estimate calls would.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import abi
from .clustersnapshot import ClusterSnapshot, NodeInfo
from .k8s import Pod
from .predicatechecker import SchedulerBasedPredicateChecker, unsupported
from .scope import UnsupportedByKernels, out_of_scope_reason

BinpackingEstimatorName = "binpacking"          # estimator.go:27-28
__all__ = ["BinpackingNodeEstimator", "UnsupportedByKernels", "estimate_batch"]


@dataclass
class ThresholdBasedEstimationLimiter:
    max_nodes: int = 0
    max_duration: float = 0.0

    def __post_init__(self):
        if self.max_duration:
            raise ValueError("maxDuration > 0 makes Estimate non-deterministic (threshold_based_limiter.go:46-47); "
                             "the device limiter implements the node cap only")


def NewThresholdBasedEstimationLimiter(max_nodes: int, max_duration: float = 0.0):  # noqa: N802
    return ThresholdBasedEstimationLimiter(max_nodes, max_duration)


class BinpackingNodeEstimator:
    def __init__(self, predicate_checker: SchedulerBasedPredicateChecker, cluster_snapshot: ClusterSnapshot,
                 limiter: ThresholdBasedEstimationLimiter):
        self.predicate_checker = predicate_checker
        self.cluster_snapshot = cluster_snapshot
        self.limiter = limiter
        self.last_result = None

    def Estimate(self, pods: list, node_template: NodeInfo, node_group=None):  # noqa: N802
        counts, scheduled = estimate_batch(self.predicate_checker, self.cluster_snapshot, [(pods, node_template)],
                                           self.limiter)
        return counts[0], scheduled[0]


def NewBinpackingNodeEstimator(predicate_checker, cluster_snapshot, limiter):  # noqa: N802
    return BinpackingNodeEstimator(predicate_checker, cluster_snapshot, limiter)


def estimate_batch(checker: SchedulerBasedPredicateChecker, snapshot: ClusterSnapshot, groups: list,
                   limiter: ThresholdBasedEstimationLimiter):
    """Estimate for [(pods, template NodeInfo)] in order; returns (counts, scheduled pod lists)."""
    all_pods: list[Pod] = []
    offs = [0]
    for pods, _ in groups:
        all_pods.extend(pods)
        offs.append(len(all_pods))
    templates_api = [(t.node, list(t.pods)) for _, t in groups]
    snapshot.ensure(pods=all_pods, templates=templates_api)
    table = snapshot.interner.encode_pods(all_pods)
    templates = np.zeros(len(groups), abi.TEMPLATE_DTYPE)
    for g, (node, tpods) in enumerate(templates_api):
        templates[g] = snapshot.interner.encode_template(node, tpods)
    pod_idx = np.arange(len(all_pods), dtype=np.int32)
    with unsupported("Estimate: the snapshot holds a pod with required anti-affinity"):
        out = snapshot.backend.estimate(table, np.array(offs, np.int32), pod_idx, templates, limiter.max_nodes,
                                        checker.last_index)
    counts, scheduled = [], []
    for g in range(len(groups)):
        r = out.results[g]
        if int(r["status"]) == abi.CA_EUNSUPPORTED:
            why = next((out_of_scope_reason(p) for p in groups[g][0] if out_of_scope_reason(p)), None)
            raise UnsupportedByKernels(f"node group {g}: " + (why or "pods depend on node identity (hostname / "
                                                                      "nodeName) or template pods need InterPodAffinity"))
        counts.append(int(r["node_count"]))
        n = int(r["n_scheduled"])
        scheduled.append([all_pods[i] for i in out.sched_pod[offs[g]: offs[g] + n]])
        checker.evals += int(r["evals"])
    checker.last_index = out.last_index
    return counts, scheduled
