"""ClusterSnapshot over a mirror backend (the MI355X ``ca_mirror`` by default).

Mirrors CA/simulator/clustersnapshot/clustersnapshot.go:29-55 (AddNode, AddNodes,
AddNodeWithPods, AddPod, RemovePod, Fork, Revert, Commit, Clear, NodeInfos) and
WithForkedSnapshot (:62-79).  Node order is the canonical order of SURVEY.md fact 2:
AddNode order, nodes added in a fork appended.

The facade keeps the API objects it was given and an operation log since Clear()
(fork markers included).  When a new object needs an id that is not interned yet
(a new label pair, port triple, taint class...), every record is re-encoded and the
log is replayed into the backend, so one encoding always covers the whole mirror.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Optional

from . import abi
from .intern import Interner
from .k8s import Node, Pod


class NodeNotFoundError(KeyError):
    """clustersnapshot.ErrNodeNotFound (clustersnapshot.go:58)."""


@dataclass
class NodeInfo:
    """The parts of schedulerframework.NodeInfo the path reads."""
    node: Node
    pods: list = field(default_factory=list)

    def Node(self) -> Node:  # noqa: N802 - reference spelling
        return self.node


class _State:
    def __init__(self):
        self.names: list[str] = []
        self.pos: dict[str, int] = {}
        self.nodes: dict[str, Node] = {}
        self.pods: dict[str, list] = {}            # node name -> [(Pod, mirror id)] in NodeInfo.Pods order

    def add_node(self, n: Node) -> None:
        if n.name in self.pos:
            raise ValueError(f"node {n.name} already in snapshot")
        self.pos[n.name] = len(self.names)
        self.names.append(n.name)
        self.nodes[n.name] = n
        self.pods[n.name] = []

    def add_pod(self, p: Pod, node: str, pid: int) -> None:
        self.pods[node].append((p, pid))

    def remove_node(self, name: str) -> None:
        self.names.remove(name)
        self.pos = {n: i for i, n in enumerate(self.names)}
        del self.nodes[name]
        del self.pods[name]

    def remove_pod(self, ns: str, name: str, node: str) -> int:
        lst = self.pods[node]
        for i, (p, pid) in enumerate(lst):
            if p.namespace == ns and p.name == name:
                lst[i] = lst[-1]                   # swap-with-last (SF/types.go:660-663)
                lst.pop()
                return pid
        raise KeyError(f"pod {ns}/{name} not on node {node}")


class ClusterSnapshot:
    def __init__(self, backend=None):
        if backend is None:
            from .native import Mirror
            backend = Mirror(0)
        self.backend = backend
        self.interner = Interner()
        self._log: list = []
        self._state = _State()
        self._stack: list[_State] = []

    # -- encoding / replay ------------------------------------------------------
    def _sizes(self):
        i = self.interner
        return tuple((len(u), len(u.overflow)) for u in (i.taints, i.pairs, i.keys, i.int_keys, i.ports, i.scalars)) + \
            (len(i.port_groups_over),)

    def ensure(self, nodes=(), pods=(), templates=()) -> None:
        """Intern new objects; re-encode and replay when a universe grew."""
        before = self._sizes()
        self.interner.observe(nodes, pods, templates)
        if self._sizes() != before and self._log:
            self._replay()

    def _replay(self) -> None:
        log = self._log
        self._log = []
        self._state = _State()
        self._stack = []
        self.backend.clear()
        for op in log:
            self._apply(op)

    def _apply(self, op) -> None:
        kind = op[0]
        st = self._state
        if kind == "node":
            rec = self.interner.encode_nodes([op[1]])
            st.add_node(op[1])
            self.backend.add_nodes(rec)
        elif kind == "pod":
            pod, node = op[1], op[2]
            if node not in st.pos:
                raise NodeNotFoundError(node)
            table = self.interner.encode_pods([pod])
            ids = self.backend.add_pods(table, [0], [st.pos[node]])
            st.add_pod(pod, node, int(ids[0]))
        elif kind == "rmpod":
            pid = st.remove_pod(op[1], op[2], op[3])
            self.backend.remove_pod(pid)
        elif kind == "rmnode":
            pos = st.pos[op[1]]
            self.backend.remove_node(pos)
            st.remove_node(op[1])
        elif kind == "fork":
            self._stack.append(copy.deepcopy(st))
            self.backend.fork()
        self._log.append(op)

    # -- ClusterSnapshot interface ------------------------------------------------
    def AddNode(self, node: Node) -> None:  # noqa: N802
        self.ensure(nodes=[node])
        self._apply(("node", node))

    def AddNodes(self, nodes: list) -> None:  # noqa: N802
        self.ensure(nodes=nodes)
        for n in nodes:
            self._apply(("node", n))

    def AddPod(self, pod: Pod, node_name: str) -> None:  # noqa: N802
        if node_name not in self._state.pos:
            raise NodeNotFoundError(node_name)
        self.ensure(pods=[pod])
        self._apply(("pod", pod, node_name))

    def AddNodeWithPods(self, node: Node, pods: list) -> None:  # noqa: N802
        self.ensure(nodes=[node], pods=pods)
        self._apply(("node", node))
        for p in pods:
            self._apply(("pod", p, node.name))

    def RemovePod(self, namespace: str, name: str, node_name: str) -> None:  # noqa: N802
        if node_name not in self._state.pos:
            raise NodeNotFoundError(node_name)
        self._apply(("rmpod", namespace, name, node_name))

    def RemoveNode(self, node_name: str) -> None:  # noqa: N802
        """RemoveNode (clustersnapshot.go:38; delta.go:150-186): the node and its pods leave."""
        if node_name not in self._state.pos:
            raise NodeNotFoundError(node_name)
        self._apply(("rmnode", node_name))

    def Fork(self) -> None:  # noqa: N802
        self._apply(("fork",))

    def Revert(self) -> None:  # noqa: N802
        if not self._stack:
            raise RuntimeError("Revert without Fork")
        self.backend.revert()
        self._state = self._stack.pop()
        i = max(i for i, op in enumerate(self._log) if op[0] == "fork")
        del self._log[i:]

    def Commit(self) -> None:  # noqa: N802
        if not self._stack:
            raise RuntimeError("Commit without Fork")
        self.backend.commit()
        self._stack.pop()
        i = max(i for i, op in enumerate(self._log) if op[0] == "fork")
        del self._log[i]

    def Clear(self) -> None:  # noqa: N802
        self.backend.clear()
        self._log = []
        self._state = _State()
        self._stack = []
        self.interner = Interner()

    def record_added_pods(self, placed: list) -> None:
        """Pods the backend already added (a batched AddPod, e.g. FilterOutSchedulable):
        [(pod, node name, mirror pod id)] — recorded as AddPod ops without re-applying them."""
        st = self._state
        for pod, node, pid in placed:
            st.add_pod(pod, node, int(pid))
            self._log.append(("pod", pod, node))

    def record_moves(self, groups: list) -> None:
        """Moves the backend already committed (the planner, ca_plan_removals), recorded as
        the ops findPlaceFor + Commit performs (cluster.go:228-242): per removed candidate,
        RemovePod of every pod to move, then AddPod of each copy on its destination.
        groups: [(candidate node name, [(pod, copy, destination name, copy's mirror id)])]."""
        st = self._state
        for node, moves in groups:
            for pod, _, _, _ in moves:
                st.remove_pod(pod.namespace, pod.name, node)
                self._log.append(("rmpod", pod.namespace, pod.name, node))
            for _, cp, dest, pid in moves:
                st.add_pod(cp, dest, int(pid))
                self._log.append(("pod", cp, dest))

    # -- NodeInfos() lister ----------------------------------------------------
    def List(self) -> list:  # noqa: N802
        st = self._state
        return [NodeInfo(st.nodes[n], [p for p, _ in st.pods[n]]) for n in st.names]

    def Get(self, name: str) -> NodeInfo:  # noqa: N802
        st = self._state
        if name not in st.pos:
            raise NodeNotFoundError(name)
        return NodeInfo(st.nodes[name], [p for p, _ in st.pods[name]])

    # -- helpers for the simulators ------------------------------------------------
    def node_names(self) -> list[str]:
        return list(self._state.names)

    def position(self, name: str) -> int:
        if name not in self._state.pos:
            raise NodeNotFoundError(name)
        return self._state.pos[name]

    def name_at(self, pos: int) -> str:
        return self._state.names[pos]

    def pod_ids(self, node_name: str) -> list:
        return list(self._state.pods[node_name])

    def encode(self, pods: list) -> abi.PodTable:
        self.ensure(pods=pods)
        return self.interner.encode_pods(pods)


def with_forked_snapshot(snapshot: ClusterSnapshot, f, persist: bool = False):
    """WithForkedSnapshot (clustersnapshot.go:62-79)."""
    snapshot.Fork()
    err = None
    try:
        err = f()
    finally:
        if err is None and persist:
            snapshot.Commit()
        else:
            snapshot.Revert()
    return err
