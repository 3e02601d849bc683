"""SchedulerBasedPredicateChecker over the mirror (CA/simulator/predicatechecker).

FitsAnyNode / FitsAnyNodeMatching / CheckPredicates with the reference's
semantics (schedulerbased.go:83-185): the rotating scan keeps ``last_index`` on
the checker object and shares it with every caller, and CheckPredicates returns
a PredicateError whose message strings match error.go:24-107 and the plugins'
reason constants.
"""
from __future__ import annotations

import contextlib
from typing import Callable, Optional, Union

import numpy as np

from . import abi
from .clustersnapshot import ClusterSnapshot, NodeInfo, NodeNotFoundError
from .k8s import Pod
from .scope import UnsupportedByKernels


@contextlib.contextmanager
def unsupported(what: str):
    """Map a backend's CA_EUNSUPPORTED (include/casim.h kernel scope) to UnsupportedByKernels."""
    try:
        yield
    except Exception as e:                      # CasimError (libcasim) / OracleError (checker)
        if getattr(e, "status", None) == abi.CA_EUNSUPPORTED:
            raise UnsupportedByKernels(what) from e
        raise

NotSchedulablePredicateError = 0     # error.go:27-32
InternalPredicateError = 1

ERR_REASON_UNSCHEDULABLE = "node(s) were unschedulable"                           # node_unschedulable.go:44
ERR_REASON_NODE_NAME = "node(s) didn't match the requested node name"              # node_name.go:39
ERR_REASON_AFFINITY = "node(s) didn't match Pod's node affinity/selector"          # node_affinity.go:59
ERR_REASON_AFFINITY_CONFLICT = "pod affinity terms conflict"                       # node_affinity.go:65
ERR_REASON_PORTS = "node(s) didn't have free ports for the requested pod ports"    # node_ports.go:45


class SchedulingError(Exception):
    pass


class PredicateError:
    """predicatechecker.PredicateError (error.go:35-107)."""

    def __init__(self, error_type: int, predicate_name: str, message: str, reasons: list, debug_info=None):
        self.error_type = error_type
        self.predicate_name = predicate_name
        self.error_message = message
        self.reasons = list(reasons or [])
        self.debug_info = debug_info or (lambda: "")

    def ErrorType(self) -> int:  # noqa: N802
        return self.error_type

    def PredicateName(self) -> str:  # noqa: N802
        return self.predicate_name

    def Message(self) -> str:  # noqa: N802
        return self.error_message or "unknown error"

    def VerboseMessage(self) -> str:  # noqa: N802
        return "%s; predicateName=%s; reasons: %s; debugInfo=%s" % (
            self.Message(), self.predicate_name, ", ".join(self.reasons), self.debug_info())

    def Reasons(self) -> list:  # noqa: N802
        return self.reasons

    def __repr__(self) -> str:
        return f"PredicateError({self.VerboseMessage()!r})"


NodeMatcher = Union[None, Callable[[NodeInfo], bool], set, frozenset]


def _go_taints(taints) -> str:
    inner = ", ".join('v1.Taint{Key:"%s", Value:"%s", Effect:"%s", TimeAdded:<nil>}' % (t.key, t.value, t.effect)
                      for t in taints)
    return "[]v1.Taint{" + inner + "}"


class SchedulerBasedPredicateChecker:
    def __init__(self):
        self.last_index = 0          # schedulerbased.go:43
        self.evals = 0               # RunFilterPlugins calls (metric)

    # -- closure -> match spec ------------------------------------------------
    @staticmethod
    def _match(snapshot: ClusterSnapshot, node_matches: NodeMatcher):
        if node_matches is None:
            return (abi.CA_MATCH_ALL, 0, 0, -1, None)
        names = snapshot.node_names()
        if isinstance(node_matches, (set, frozenset)):
            mask = np.array([n in node_matches for n in names], np.uint8)
        else:
            infos = snapshot.List()
            mask = np.array([bool(node_matches(ni)) for ni in infos], np.uint8)
        return (abi.CA_MATCH_MASK, 0, 0, -1, mask)

    def FitsAnyNode(self, snapshot: Optional[ClusterSnapshot], pod: Pod):  # noqa: N802
        return self.FitsAnyNodeMatching(snapshot, pod, None)

    def FitsAnyNodeMatching(self, snapshot: Optional[ClusterSnapshot], pod: Pod, node_matches: NodeMatcher = None):  # noqa: N802
        if snapshot is None:
            return "", SchedulingError("ClusterSnapshot not provided")
        table = snapshot.encode([pod])
        match = self._match(snapshot, node_matches)
        with unsupported(f"FitsAnyNode({pod.name}): out of kernel scope"):
            node, li, pf, ev = snapshot.backend.fits_any_node(table, 0, match, self.last_index)
        self.evals += ev
        if pf:
            return "", SchedulingError(f"error running pre filter plugins for pod {pod.name}; {ERR_REASON_AFFINITY_CONFLICT}")
        if node < 0:
            return "", SchedulingError(f"cannot put pod {pod.name} on any node")
        self.last_index = li
        return snapshot.name_at(node), None

    def CheckPredicates(self, snapshot: Optional[ClusterSnapshot], pod: Pod, node_name: str):  # noqa: N802
        if snapshot is None:
            return PredicateError(InternalPredicateError, "", "ClusterSnapshot not provided", None)
        try:
            pos = snapshot.position(node_name)
        except NodeNotFoundError as e:
            return PredicateError(InternalPredicateError, "",
                                  f"Error obtaining NodeInfo for name {node_name}; {e}", None)
        table = snapshot.encode([pod])
        with unsupported(f"CheckPredicates({pod.name}): out of kernel scope"):
            typ, plugin, reasons, taint = snapshot.backend.check_predicates(table, 0, pos)
        if typ == abi.CA_PRED_INTERNAL:
            return PredicateError(InternalPredicateError, "", ERR_REASON_AFFINITY_CONFLICT,
                                  [ERR_REASON_AFFINITY_CONFLICT])
        self.evals += 1                                  # RunFilterPlugins ran (:171)
        if typ == abi.CA_PRED_OK:
            return None
        node = snapshot.Get(node_name).node
        name = abi.PLUGIN_NAMES[plugin]
        debug = None
        if plugin == abi.CA_PLUGIN_NODE_UNSCHEDULABLE:
            rs = [ERR_REASON_UNSCHEDULABLE]
        elif plugin == abi.CA_PLUGIN_NODE_NAME:
            rs = [ERR_REASON_NODE_NAME]
        elif plugin == abi.CA_PLUGIN_TAINT_TOLERATION:
            # first untolerated NoSchedule/NoExecute taint in node order (helpers.go:78-88)
            from .intern import tolerates
            t = next(t for t in node.taints if t.effect in ("NoSchedule", "NoExecute")
                     and not any(tolerates(x, t) for x in pod.tolerations))
            rs = ["node(s) had untolerated taint {%s: %s}" % (t.key, t.value)]
            taints = list(node.taints)
            debug = lambda: "taints on node: " + _go_taints(taints)  # noqa: E731
        elif plugin == abi.CA_PLUGIN_NODE_AFFINITY:
            rs = [ERR_REASON_AFFINITY]
        elif plugin == abi.CA_PLUGIN_NODE_PORTS:
            rs = [ERR_REASON_PORTS]
        else:
            rs = []
            if reasons & abi.CA_REASON_TOO_MANY_PODS:
                rs.append("Too many pods")
            if reasons & abi.CA_REASON_INSUFF_CPU:
                rs.append("Insufficient cpu")
            if reasons & abi.CA_REASON_INSUFF_MEMORY:
                rs.append("Insufficient memory")
            if reasons & abi.CA_REASON_INSUFF_EPHEMERAL:
                rs.append("Insufficient ephemeral-storage")
            inv = {i: n for n, i in snapshot.interner.scalars.ids.items()}
            for i in range(abi.CA_MAX_SCALAR):
                if reasons & (abi.CA_REASON_INSUFF_SCALAR0 << i):
                    rs.append(f"Insufficient {inv.get(i, i)}")
        return PredicateError(NotSchedulablePredicateError, name, ", ".join(rs), rs, debug)
