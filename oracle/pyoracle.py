"""ctypes binding of the CPU restatement (oracle/casim_oracle.c).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py as the checker.  It exposes the same methods as
``autoscaler_amd.native.Mirror`` so a parity test can drive both with one script.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from autoscaler_amd import abi
from autoscaler_amd.abi import ptr
from autoscaler_amd.native import EstimateOutput, FilterOutput, PlanOutput, RemovalOutput, filter_args, plan_args

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libcasim_oracle.so")
_LIB = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def load() -> C.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    vp, i32, p = C.c_void_p, C.c_int32, C.POINTER
    sigs = {
        "or_create": ([], vp), "or_destroy": ([vp], None), "or_clear": ([vp], C.c_int),
        "or_add_nodes": ([vp, vp, i32, p(i32)], C.c_int),
        "or_add_pods": ([vp, vp, vp, vp, i32, vp], C.c_int),
        "or_remove_pod": ([vp, i32], C.c_int),
        "or_remove_node": ([vp, i32], C.c_int),
        "or_scope_blockers": ([vp], C.c_int),
        "or_set_sort_mode": ([vp, i32], C.c_int),
        "go_sort_slice_desc": ([vp, i32, vp], None),
        "go_sort_slice_desc_limit": ([vp, i32, i32, vp], None),
        "go_sort_stats": ([vp], None),
        "or_fork": ([vp], C.c_int), "or_revert": ([vp], C.c_int), "or_commit": ([vp], C.c_int),
        "or_node_count": ([vp], C.c_int), "or_node_pods": ([vp, i32, vp, i32], C.c_int),
        "or_pod_node": ([vp, i32], C.c_int), "or_node_state": ([vp, i32, vp], C.c_int),
        "or_fits_any_node": ([vp, vp, i32, vp, p(i32), p(i32), p(i32), p(C.c_uint64)], C.c_int),
        "or_check_predicates": ([vp, vp, i32, i32, vp], C.c_int),
        "or_check_templates": ([vp, vp, vp, i32, vp, i32, vp], C.c_int),
        "or_node_utilization": ([vp, i32, vp, vp, i32, i32, C.c_int64, vp], C.c_int),
        "or_estimate": ([vp, vp, vp, vp, vp, i32, vp, p(i32), vp, vp, vp], C.c_int),
        "or_try_schedule_pods": ([vp, vp, i32, vp, i32, vp, p(i32), vp, p(C.c_uint64)], C.c_int),
        "or_find_nodes_to_remove": ([vp, vp, i32, vp, vp, vp, vp, vp, p(i32), vp, vp], C.c_int),
        "or_plan_removals": ([vp, vp, i32, vp, vp, vp, vp, i32, vp, vp, i32, p(i32), vp, vp, i32, p(i32)], C.c_int),
        "or_filter_out_schedulable": ([vp, vp, vp, i32, vp, i32, vp, p(i32), vp, vp, p(i32), p(C.c_uint64), p(i32)],
                                      C.c_int),
    }
    for name, (args, res) in sigs.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    _LIB = lib
    return lib


class OracleError(RuntimeError):
    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(f"oracle {what}: status {status}")


def _check(st: int, what: str) -> None:
    if st != abi.CA_OK:
        raise OracleError(st, what)


class OracleState:
    backend_name = "oracle"

    def __init__(self):
        self.lib = load()
        self.h = self.lib.or_create()

    def close(self) -> None:
        if self.h:
            self.lib.or_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def clear(self) -> None:
        _check(self.lib.or_clear(self.h), "clear")

    def add_nodes(self, nodes: np.ndarray) -> int:
        nodes = np.ascontiguousarray(nodes, dtype=abi.NODE_DTYPE)
        first = C.c_int32(0)
        _check(self.lib.or_add_nodes(self.h, ptr(nodes), len(nodes), C.byref(first)), "add_nodes")
        return first.value

    def add_pods(self, table: abi.PodTable, idx, node_pos) -> np.ndarray:
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        node_pos = np.ascontiguousarray(node_pos, dtype=np.int32)
        out = np.zeros(len(idx), np.int32)
        _check(self.lib.or_add_pods(self.h, table.ref, ptr(idx), ptr(node_pos), len(idx), ptr(out)), "add_pods")
        return out

    def remove_pod(self, pod_id: int) -> None:
        _check(self.lib.or_remove_pod(self.h, pod_id), "remove_pod")

    def remove_node(self, pos: int) -> None:
        _check(self.lib.or_remove_node(self.h, pos), "remove_node")

    def scope_blockers(self) -> int:
        return self.lib.or_scope_blockers(self.h)

    def set_sort_mode(self, mode: str) -> None:
        """Estimate's score sort: "stable" (the device order) or "go" (Go 1.19 sort.Slice)."""
        _check(self.lib.or_set_sort_mode(self.h, {"stable": 0, "go": 1}[mode]), "set_sort_mode")

    def fork(self) -> None:
        _check(self.lib.or_fork(self.h), "fork")

    def revert(self) -> None:
        _check(self.lib.or_revert(self.h), "revert")

    def commit(self) -> None:
        _check(self.lib.or_commit(self.h), "commit")

    def node_count(self) -> int:
        return self.lib.or_node_count(self.h)

    def pod_node(self, pod_id: int) -> int:
        return self.lib.or_pod_node(self.h, pod_id)

    def node_pods(self, node: int) -> list[int]:
        out = np.zeros(4096, np.int32)
        n = self.lib.or_node_pods(self.h, node, ptr(out), len(out))
        return out[: max(n, 0)].tolist()

    def node_state(self, node: int) -> tuple[int, int, int, int]:
        out = np.zeros(4, np.int64)
        _check(self.lib.or_node_state(self.h, node, ptr(out)), "node_state")
        return tuple(int(x) for x in out)

    def fits_any_node(self, table: abi.PodTable, pod: int, match=None, last_index: int = 0):
        ms, mask = abi.match_spec(*(match or ()))
        li = C.c_int32(last_index)
        out = C.c_int32(-1)
        pf = C.c_int32(0)
        ev = C.c_uint64(0)
        _check(self.lib.or_fits_any_node(self.h, table.ref, pod, C.byref(ms), C.byref(li), C.byref(out),
                                         C.byref(pf), C.byref(ev)), "fits_any_node")
        del mask
        return out.value, li.value, pf.value, ev.value

    def check_predicates(self, table: abi.PodTable, pod: int, node: int):
        r = abi.PredResultC()
        _check(self.lib.or_check_predicates(self.h, table.ref, pod, node, C.byref(r)), "check_predicates")
        return r.type, r.plugin, r.reasons, r.taint

    def check_templates(self, table: abi.PodTable, samples, templates: np.ndarray) -> np.ndarray:
        """ComputeExpansionOption's CheckPredicates(sample, template copy) matrix [G][E]."""
        sm = np.ascontiguousarray(samples, dtype=np.int32)
        tm = np.ascontiguousarray(templates, dtype=abi.TEMPLATE_DTYPE)
        out = np.zeros((len(tm), len(sm)), abi.PRED_RESULT_DTYPE)
        _check(self.lib.or_check_templates(self.h, table.ref, ptr(sm), len(sm), ptr(tm), len(tm), ptr(out)),
               "check_templates")
        return out

    def estimate(self, table: abi.PodTable, group_off, pod_idx, templates: np.ndarray, max_nodes: int,
                 last_index: int = 0) -> EstimateOutput:
        off = np.ascontiguousarray(group_off, dtype=np.int32)
        idx = np.ascontiguousarray(pod_idx, dtype=np.int32)
        tm = np.ascontiguousarray(templates, dtype=abi.TEMPLATE_DTYPE)
        total = int(off[-1]) if len(off) else 0
        res = np.zeros(len(tm), abi.ESTIMATE_RESULT_DTYPE)
        sp = np.full(max(total, 1), -1, np.int32)
        sn = np.full(max(total, 1), -1, np.int32)
        lim = abi.LimiterC(max_nodes, 0)
        li = C.c_int32(last_index)
        _check(self.lib.or_estimate(self.h, table.ref, ptr(off), ptr(idx), ptr(tm), len(tm), C.byref(lim),
                                    C.byref(li), ptr(res), ptr(sp), ptr(sn)), "estimate")
        return EstimateOutput(res, sp[:total], sn[:total], li.value)

    def try_schedule_pods(self, pod_ids, match, break_on_failure: bool, hints, last_index: int = 0):
        ids = np.ascontiguousarray(pod_ids, dtype=np.int32)
        ms, mask = abi.match_spec(*match)
        hints = np.array(hints, dtype=np.int32, copy=True)
        dest = np.full(max(len(ids), 1), -1, np.int32)
        li = C.c_int32(last_index)
        ev = C.c_uint64(0)
        placed = self.lib.or_try_schedule_pods(self.h, ptr(ids), len(ids), C.byref(ms), int(break_on_failure),
                                               ptr(hints), C.byref(li), ptr(dest), C.byref(ev))
        del mask
        return placed, dest[: len(ids)], hints, li.value, ev.value

    def filter_out_schedulable(self, table: abi.PodTable, order=None, class_owner=None, hints=None,
                               last_index: int = 0, podset=None) -> FilterOutput:
        del podset                                      # device residency: the mirror only
        a = filter_args(table, order, class_owner, hints)
        li = C.c_int32(last_index)
        ev = C.c_uint64(0)
        ov = C.c_int32(0)
        placed = C.c_int32(0)
        _check(self.lib.or_filter_out_schedulable(self.h, table.ref, ptr(a.order), a.n, a.owner_ptr, a.n_classes,
                                                  ptr(a.hints), C.byref(li), ptr(a.node), ptr(a.pod_id),
                                                  C.byref(ov), C.byref(ev), C.byref(placed)), "filter_out_schedulable")
        return a.output(placed.value, li.value, ev.value, ov.value)

    def find_nodes_to_remove(self, candidates, dest_mask, cand_status, move_off, move_pods, hints,
                             last_index: int = 0) -> RemovalOutput:
        cand = np.ascontiguousarray(candidates, dtype=np.int32)
        mask = np.ascontiguousarray(dest_mask, dtype=np.uint8)
        status = np.ascontiguousarray(cand_status if cand_status is not None else np.zeros(len(cand)), dtype=np.int32)
        off = np.ascontiguousarray(move_off, dtype=np.int32)
        moves = np.ascontiguousarray(move_pods, dtype=np.int32)
        hints = np.array(hints, dtype=np.int32, copy=True)
        res = np.zeros(len(cand), abi.REMOVAL_RESULT_DTYPE)
        dest = np.full(max(len(moves), 1), -1, np.int32)
        li = C.c_int32(last_index)
        _check(self.lib.or_find_nodes_to_remove(self.h, ptr(cand), len(cand), ptr(mask), ptr(status), ptr(off),
                                                ptr(moves), ptr(hints), C.byref(li), ptr(res), ptr(dest)),
               "find_nodes_to_remove")
        return RemovalOutput(res, dest[: len(moves)], hints, li.value)

    def plan_removals(self, candidates, dest_mask, cand_status, move_off, move_pods, hints, last_index: int = 0,
                      max_removable: int = 0, pdb_allowed=None, pdb_pod_off=None, pdb_pod=None) -> PlanOutput:
        a = plan_args(candidates, dest_mask, cand_status, move_off, move_pods, hints, pdb_allowed, pdb_pod_off, pdb_pod)
        li = C.c_int32(last_index)
        nm = C.c_int32(0)
        _check(self.lib.or_plan_removals(self.h, ptr(a.cand), len(a.cand), ptr(a.mask), ptr(a.status), ptr(a.off),
                                         ptr(a.moves), int(max_removable), a.pdb_ptr, ptr(a.hints), len(a.hints),
                                         C.byref(li), ptr(a.res), ptr(a.out_moves), len(a.out_moves), C.byref(nm)),
               "plan_removals")
        if nm.value > len(a.out_moves):     # (the commits are made: a bigger buffer cannot re-run them)
            raise OracleError(abi.CA_ECAPACITY, "plan_removals moves")
        a.res = a.res[: len(a.cand)]
        return a.output(li.value, nm.value)


def go_sort_desc(keys, limit: int = 0) -> np.ndarray:
    """Go 1.19 sort.Slice(x, key[i] > key[j]) (oracle/gosort.c): the permutation.  limit > 0
    replaces the initial recursion limit bits.Len(n) (reaches the heapSort fallback)."""
    k = np.ascontiguousarray(keys, dtype=np.float64)
    perm = np.zeros(max(len(k), 1), np.int32)
    load().go_sort_slice_desc_limit(ptr(k), len(k), int(limit), ptr(perm))
    return perm[: len(k)]


def go_sort_stats() -> tuple:
    out = np.zeros(2, np.int64)
    load().go_sort_stats(ptr(out))
    return int(out[0]), int(out[1])


def node_utilization(nodes: np.ndarray, pod_off: np.ndarray, pods: np.ndarray, skip_daemonset_pods: bool,
                     skip_mirror_pods: bool, now_ns: int) -> np.ndarray:
    """or_node_utilization: utilization.Calculate + the FindEmptyNodesToRemove verdict per node."""
    nodes = np.ascontiguousarray(nodes, abi.UTIL_NODE_DTYPE)
    pod_off = np.ascontiguousarray(pod_off, np.int32)
    pods = np.ascontiguousarray(pods, abi.UTIL_POD_DTYPE)
    out = np.zeros(len(nodes), abi.UTIL_INFO_DTYPE)
    _check(load().or_node_utilization(ptr(nodes), len(nodes), ptr(pod_off), ptr(pods), int(skip_daemonset_pods),
                                      int(skip_mirror_pods), int(now_ns), ptr(out)), "node_utilization")
    return out


def runonce_cpu_util(ui, now_ns: int):
    """The CPU port's utilization step of autoscaler_amd.runonce.run (or_node_utilization
    over the UtilInput's full rows): the parity checker and the bench's CPU baseline."""
    return node_utilization(ui.nodes, ui.off, ui.pods, False, False, now_ns)
