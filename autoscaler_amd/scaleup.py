"""ScaleUp's option computation for every node group in one pass (CA/core/scaleup).

The reference computes, per node group (orchestrator.go:139-178 -> ComputeExpansionOption
:443-491): Fork; add the template node with its pods; CheckPredicates(sample pod of
every pod equivalence group, template node); Revert; then Estimate(pods of the
groups that passed, template).  Here:

* ``BuildPodGroups`` (equivalence/groups.go:38-102) stays on the host: pods grouped by
  controller UID + equal labels and spec, at most 10 groups per controller, pods
  without a controller (or DaemonSet pods) alone;
* the feasibility of every (node group, pod group) pair is one device call
  (``ca_check_templates``: CheckPredicates of the sample on a fresh template copy,
  schedulerbased.go:139-185 results, reasons included for eg.SchedulingErrors);
* the options' Estimates are one batch (``estimate_batch``: shared lastIndex, exactly
  as the reference's consecutive Estimate calls).

Order: the reference ranges over BuildPodGroups' map (random order in Go); groups
here are in first-occurrence order, so an option's pods are in a canonical order
(Estimate's tie order).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import abi
from .clustersnapshot import ClusterSnapshot, NodeInfo
from .estimator import ThresholdBasedEstimationLimiter, estimate_batch
from .k8s import Pod, is_daemonset_pod
from .predicatechecker import SchedulerBasedPredicateChecker
from .simulator import SimilarPodsScheduling

MAX_EQUIVALENCE_GROUPS_BY_CONTROLLER = 10          # groups.go:57


@dataclass
class PodGroup:
    """equivalence.PodGroup (groups.go:30-35)."""
    pods: list
    scheduling_errors: dict = field(default_factory=dict)     # node group id -> ca_pred_result
    schedulable: bool = False


def BuildPodGroups(pods: list) -> list:  # noqa: N802
    """groupPodsBySchedulingProperties (groups.go:59-102), groups in first-occurrence order."""
    groups: list[PodGroup] = []
    by_controller: dict = {}
    for pod in pods:
        ref = pod.controller_ref()
        if ref is None or is_daemonset_pod(pod):                  # :68-72 (pod_util.IsDaemonSetPod)
            groups.append(PodGroup([pod]))
            continue
        egs = by_controller.setdefault(ref.uid, [])
        sig = SimilarPodsScheduling._sig(pod)                      # labels + spec equality (:105-112)
        gid = next((g for s, g in egs if s == sig), None)
        if gid is not None:
            groups[gid].pods.append(pod)
            continue
        if len(egs) < MAX_EQUIVALENCE_GROUPS_BY_CONTROLLER:       # :79-86
            egs.append((sig, len(groups)))
        groups.append(PodGroup([pod]))
    return groups


@dataclass
class ExpansionOption:
    """expander.Option (the parts the Estimate fills): node group, count, pods."""
    node_group: object
    node_count: int
    pods: list


def ComputeExpansionOptions(snapshot: ClusterSnapshot, checker: SchedulerBasedPredicateChecker,  # noqa: N802
                            pod_groups: list, node_groups: list, limiter: ThresholdBasedEstimationLimiter):
    """ComputeExpansionOption (orchestrator.go:443-491) for every (node group, template
    NodeInfo) in ``node_groups``: pod groups' feasibility in one device call, then one
    Estimate batch over the options that got pods.  Marks pod groups schedulable and
    records their per-node-group predicate results, as the reference does."""
    samples = [g.pods[0] for g in pod_groups]
    templates_api = [(t.node, list(t.pods)) for _, t in node_groups]
    snapshot.ensure(pods=[p for g in pod_groups for p in g.pods], templates=templates_api)
    table = snapshot.interner.encode_pods(samples)
    tm = np.zeros(len(node_groups), abi.TEMPLATE_DTYPE)
    for k, (node, tpods) in enumerate(templates_api):
        tm[k] = snapshot.interner.encode_template(node, tpods)
    feas = snapshot.backend.check_templates(table, np.arange(len(samples), dtype=np.int32), tm)
    est_groups, est_index = [], []
    for k, (ng, info) in enumerate(node_groups):
        pods = []
        for e, pg in enumerate(pod_groups):
            r = feas[k, e]
            if int(r["type"]) == abi.CA_PRED_OK:
                pods.extend(pg.pods)
                pg.schedulable = True
            else:
                pg.scheduling_errors[ng] = r.copy()
        if pods:
            est_groups.append((pods, info))
            est_index.append(k)
    options = [ExpansionOption(ng, 0, []) for ng, _ in node_groups]
    if est_groups:
        counts, scheduled = estimate_batch(checker, snapshot, est_groups, limiter)
        for k, c, s in zip(est_index, counts, scheduled):
            options[k].node_count = c
            options[k].pods = s
    return options, feas


__all__ = ["PodGroup", "BuildPodGroups", "ExpansionOption", "ComputeExpansionOptions", "NodeInfo", "Pod"]
