"""Random Planner (canPersist=true) cases and a step-by-step restatement of the loop.

``plan_by_steps`` restates Planner.categorizeNodes (CA/core/scaledown/planner/planner.go:
252-296) from parts the oracle already pins: one legacy single-candidate
FindNodesToRemove (a simulation on a reverted fork) per candidate, and, when it is
removable, the commit done by hand (RemovePod of the pods to move, AddPod of their
copies with Spec.NodeName and TPU requests cleared: CA/simulator/cluster.go:225-240),
PDB budgets as RemainingPdbTracker (CA/core/scaledown/pdb/basic.go:66-95).  It checks
the oracle's ``or_plan_removals`` loop, which the GPU path is then compared against."""
from __future__ import annotations

from collections import defaultdict
from dataclasses import dataclass

import numpy as np

from autoscaler_amd import abi
from autoscaler_amd.intern import Interner
from autoscaler_amd.k8s import Quantity
from randgen import rand_cluster

TPU = "cloud-tpus.google.com/v3"


@dataclass
class PlanCase:
    node_recs: np.ndarray
    table: abi.PodTable
    node_of: np.ndarray
    cands: np.ndarray
    mask: np.ndarray
    status: np.ndarray
    off: np.ndarray
    moves: np.ndarray
    hints: np.ndarray
    L0: int
    limit: int
    allowed: np.ndarray
    pdb_off: np.ndarray
    pdb_pod: np.ndarray

    def args(self):
        return (self.cands, self.mask, self.status, self.off, self.moves)

    def load(self, b) -> None:
        b.clear()
        b.add_nodes(self.node_recs)
        b.add_pods(self.table, np.arange(len(self.table), dtype=np.int32), self.node_of)

    def plan(self, b):
        return b.plan_removals(*self.args(), self.hints, self.L0, self.limit, self.allowed, self.pdb_off,
                               self.pdb_pod)


def rand_plan_case(seed: int, n_nodes: int = 12, pods_per_node: int = 4, n_pdbs: int = 0,
                   limit: int | None = None) -> PlanCase:
    rng, nodes, scheduled, _ = rand_cluster(seed, n_nodes=n_nodes, n_pods=n_nodes * pods_per_node,
                                            pods_per_node=pods_per_node)
    for p, _ in scheduled:
        if rng.random() < 0.08:
            p.containers[0].requests[TPU] = Quantity(rng.choice([1, 2]))
    pods = [p for p, _ in scheduled]
    it = Interner(nodes, pods)
    node_recs = it.encode_nodes(nodes)
    table = it.encode_pods(pods)
    pos = {n.name: i for i, n in enumerate(nodes)}
    node_of = np.array([pos[n] for _, n in scheduled], np.int32)
    N = len(nodes)
    cands = np.array(rng.sample(range(N), rng.randint(1, N)), np.int32)
    mask = np.array([rng.random() < 0.9 for _ in nodes], np.uint8)
    status = np.array([rng.choice([0, 0, 0, 0, abi.CA_UNREMOVABLE_BLOCKED_BY_POD]) for _ in cands], np.int32)
    off, moves = [0], []
    for c in cands:
        moves.extend(i for i in range(len(pods)) if node_of[i] == c and rng.random() < 0.9)
        off.append(len(moves))
    hints = np.array([rng.choice([-1, -1, rng.randrange(N)]) for _ in pods], np.int32)
    allowed = np.array([rng.randint(0, 4) for _ in range(n_pdbs)], np.int32)
    pdb_off, pdb_pod = [0], []
    for _ in pods:
        pdb_pod.extend(sorted(rng.sample(range(n_pdbs), rng.randint(0, min(2, n_pdbs)))) if n_pdbs else [])
        pdb_off.append(len(pdb_pod))
    if limit is None:
        limit = rng.choice([0, 0, 1, 2, 3])
    return PlanCase(node_recs, table, node_of, cands, mask, status, np.array(off, np.int32),
                    np.array(moves, np.int32), hints, rng.randrange(0, 3 * N), limit, allowed,
                    np.array(pdb_off, np.int32), np.array(pdb_pod, np.int32))


def moved_record(rec: np.ndarray) -> np.ndarray:
    """The copy findPlaceFor schedules: NodeName cleared, TPU requests cleared."""
    q = rec.copy()
    q["node_name_id"] = -1
    m = int(rec["tpu_scalar_mask"])
    for i in range(abi.CA_MAX_SCALAR):
        if (m >> i) & 1:
            q["req_scalar"][i] = 0
    if not (int(rec["flags"]) & abi.CA_POD_HAS_NONTPU_SCALAR_KEYS):
        q["flags"] = int(q["flags"]) & ~abi.CA_POD_HAS_SCALAR_KEYS
    return q


def plan_by_steps(o, case: PlanCase) -> dict:
    """The planner loop from single-candidate legacy sweeps + commits by hand, on oracle state o."""
    t = case.table
    recs = [t.pods[i].copy() for i in range(len(t))]
    H = case.hints.astype(np.int32).copy()
    origin = list(range(len(t)))
    extra = defaultdict(list)
    mask = case.mask.copy()
    allowed = case.allowed.astype(np.int64).copy()
    P = len(allowed)

    def member(pod, p):
        q = origin[pod]
        return p in case.pdb_pod[case.pdb_off[q]:case.pdb_off[q + 1]].tolist()

    N = len(case.node_recs)
    L = case.L0
    removed, cut = 0, False
    res = np.zeros(len(case.cands), abi.PLAN_RESULT_DTYPE)
    log = []
    for ci, node in enumerate(case.cands.tolist()):
        r = res[ci]
        r["last_index_in"] = L
        r["first_move"] = len(log)
        r["blocking_pod"] = -1
        if cut or (case.limit > 0 and removed >= case.limit):                  # planner.go:268-271
            r["reason"] = abi.CA_UNREMOVABLE_NOT_RUN
            cut = True
            continue
        lst = case.moves[case.off[ci]:case.off[ci + 1]].tolist() + extra[node]
        if not (0 <= node < N and mask[node]):
            r["reason"] = abi.CA_UNREMOVABLE_UNEXPECTED_ERROR
            continue
        if case.status[ci]:
            r["reason"] = case.status[ci]
            continue
        blocking = -1
        for p in range(P):                                                      # drain.go:73-90
            if allowed[p] >= 1:
                continue
            blocking = next((pod for pod in lst if member(pod, p)), -1)
            if blocking >= 0:
                break
        if blocking >= 0:
            r["reason"] = abi.CA_UNREMOVABLE_BLOCKED_BY_POD
            r["blocking_pod"] = blocking
            continue
        one = o.find_nodes_to_remove(np.array([node], np.int32), mask, np.zeros(1, np.int32),
                                     np.array([0, len(lst)], np.int32), np.array(lst, np.int32), H, L)
        sr = one.results[0]
        H, L = one.hints.copy(), one.last_index
        r["n_placed"] = sr["n_placed"]
        r["evals"] = sr["evals"]
        if not sr["removable"]:
            r["reason"] = abi.CA_UNREMOVABLE_NO_PLACE
            continue
        r["removable"] = 1
        r["n_moves"] = len(lst)
        for pod in lst:                                                         # cluster.go:228-233
            o.remove_pod(pod)
        for pod, dest in zip(lst, one.dest.tolist()):                           # AddPod of the copies
            q = moved_record(recs[pod])
            nid = int(o.add_pods(abi.PodTable(q[None], t.terms, t.reqs, t.names), [0], [dest])[0])
            assert nid == len(recs)
            recs.append(q)
            H = np.append(H, np.int32(dest))
            origin.append(origin[pod])
            extra[dest].append(nid)
            log.append((ci, pod, nid, dest))
        mask[node] = 0
        removed += 1
        for p in range(P):                                                      # basic.go:66-84
            count = 0
            for pod in lst:
                if member(pod, p):
                    count += 1
                    if allowed[p] < count:
                        r["risky"] = 1
        for p in range(P):                                                      # basic.go:86-95
            allowed[p] -= sum(1 for pod in lst if member(pod, p))
    moves = np.array(log, np.int32).reshape(-1, 4)
    out = np.zeros(len(moves), abi.PLAN_MOVE_DTYPE)
    for k, name in enumerate(("candidate", "pod", "new_pod", "node")):
        out[name] = moves[:, k]
    return {"results": res, "moves": out, "hints": H[: len(t)], "last_index": L, "allowed": allowed.astype(np.int32)}


def node_states(b, n: int) -> list:
    return [(b.node_pods(i), b.node_state(i)) for i in range(n)]
