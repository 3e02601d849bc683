"""Loader and thin object wrapper of ``libcasim.so`` (the MI355X product path).

There is no fallback: if the in-tree library is missing, or no HIP device is
visible, every constructor raises.  The wrapper only marshals numpy arrays into
the C ABI of ``include/casim.h``; all simulation work happens in the library.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import abi
from .abi import ptr

_LIB = None
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libcasim.so")


class CasimError(RuntimeError):
    def __init__(self, status: int, what: str):
        self.status = status
        super().__init__(f"{what}: status {status} ({_status_string(status)})")


def _status_string(status: int) -> str:
    try:
        return load().ca_status_string(status).decode()
    except Exception:  # pragma: no cover - only while the library is unusable
        return "?"


def load() -> C.CDLL:
    """Load the in-tree libcasim.so (raises if it was not built)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = os.environ.get("CASIM_LIB_PATH", LIB_PATH)    # diagnostics builds only (Makefile: prof)
    if not os.path.exists(path):
        raise RuntimeError(f"libcasim.so not built: {path} missing (run __graft_entry__.build())")
    lib = C.CDLL(path)
    vp, i32, p = C.c_void_p, C.c_int32, C.POINTER
    sigs = {
        "ca_abi_version": ([], C.c_int),
        "ca_abi_struct_sizes": ([p(i32), i32], C.c_int),
        "ca_device_count": ([p(i32)], C.c_int),
        "ca_status_string": ([C.c_int], C.c_char_p),
        "ca_host_alloc": ([C.c_size_t, p(vp)], C.c_int),
        "ca_host_free": ([vp], C.c_int),
        "ca_mirror_create": ([i32, p(vp)], C.c_int),
        "ca_mirror_destroy": ([vp], C.c_int),
        "ca_mirror_clear": ([vp], C.c_int),
        "ca_mirror_add_nodes": ([vp, vp, i32, p(i32)], C.c_int),
        "ca_mirror_add_pods": ([vp, vp, vp, vp, i32, vp], C.c_int),
        "ca_mirror_remove_pod": ([vp, i32], C.c_int),
        "ca_mirror_remove_node": ([vp, i32], C.c_int),
        "ca_mirror_scope_blockers": ([vp, p(i32)], C.c_int),
        "ca_mirror_fork": ([vp], C.c_int),
        "ca_mirror_revert": ([vp], C.c_int),
        "ca_mirror_commit": ([vp], C.c_int),
        "ca_mirror_node_count": ([vp, p(i32)], C.c_int),
        "ca_mirror_pod_node": ([vp, i32, p(i32)], C.c_int),
        "ca_mirror_node_pods": ([vp, i32, vp, i32, p(i32)], C.c_int),
        "ca_podset_create": ([vp, vp, p(vp)], C.c_int),
        "ca_podset_destroy": ([vp], C.c_int),
        "ca_fits_any_node": ([vp, vp, i32, vp, p(i32), p(i32), p(i32), p(C.c_uint64)], C.c_int),
        "ca_check_predicates": ([vp, vp, i32, i32, vp], C.c_int),
        "ca_fits_matrix": ([vp, vp, vp], C.c_int),
        "ca_check_templates": ([vp, vp, vp, i32, vp, i32, vp, vp], C.c_int),
        "ca_expansion_plan_create": ([vp, vp, i32, p(vp)], C.c_int),
        "ca_expansion_plan_run": ([vp, vp, vp, i32, vp, vp], C.c_int),
        "ca_expansion_plan_destroy": ([vp], C.c_int),
        "ca_expansion_plan_kernel_ms": ([vp, p(C.c_float)], C.c_int),
        "ca_estimate_batch": ([vp, vp, vp, vp, vp, i32, vp, p(i32), vp, vp, vp], C.c_int),
        "ca_estimate_plan_create": ([vp, vp, vp, vp, vp, i32, p(vp)], C.c_int),
        "ca_estimate_plan_run": ([vp, vp, p(i32), vp, vp, vp], C.c_int),
        "ca_estimate_plan_run_u16": ([vp, vp, p(i32), vp, vp], C.c_int),
        "ca_estimate_plan_destroy": ([vp], C.c_int),
        "ca_estimate_plan_fetch": ([vp, vp], C.c_int),
        "ca_estimate_plan_device_results": ([vp, p(vp)], C.c_int),
        "ca_estimate_plan_stats": ([vp, p(i32), p(C.c_float), p(C.c_float), p(C.c_float)], C.c_int),
        "ca_estimate_plan_chain_info": ([vp, p(i32), p(i32)], C.c_int),
        "ca_estimate_plan_rebase": ([vp, vp, i32, p(i32)], C.c_int),
        "ca_go_sort_ranks": ([i32, vp, i32, i32, i32, vp], C.c_int),
        "ca_estimate_plan_timings": ([vp, p(C.c_float), i32], C.c_int),
        "ca_estimate_plan_set_phase_timing": ([vp, i32], C.c_int),
        "ca_estimate_plan_group_ticks": ([vp, p(C.c_uint64), i32], C.c_int),
        "ca_find_nodes_to_remove": ([vp, vp, i32, vp, vp, vp, vp, vp, p(i32), vp, vp], C.c_int),
        "ca_removal_stats": ([vp, p(i32), p(C.c_float), p(C.c_float)], C.c_int),
        "ca_removal_plan_create": ([vp, vp, i32, vp, vp, vp, vp, p(vp)], C.c_int),
        "ca_removal_plan_run": ([vp, vp, p(i32), vp, vp], C.c_int),
        "ca_removal_plan_destroy": ([vp], C.c_int),
        "ca_removal_plan_sensitive_pods": ([vp, p(C.c_int64)], C.c_int),
        "ca_removal_plan_phased": ([vp, p(i32)], C.c_int),
        "ca_removal_plan_run_phase": ([vp, vp, vp, p(i32), vp, vp], C.c_int),
        "ca_sweep_compose": ([vp, i32, i32, i32, vp, p(i32)], C.c_int),
        "ca_mirror_set_hints": ([vp, vp, i32], C.c_int),
        "ca_mirror_get_hints": ([vp, vp, i32], C.c_int),
        "ca_removal_candidate_ticks": ([vp, p(C.c_uint64), i32], C.c_int),
        "ca_removal_timings": ([vp, p(C.c_float), i32], C.c_int),
        "ca_filter_out_schedulable": ([vp, vp, vp, vp, i32, vp, i32, vp, p(i32), vp, vp, p(i32), p(C.c_uint64), p(i32)],
                                      C.c_int),
        "ca_filter_stats": ([vp, p(C.c_float), i32], C.c_int),
        "ca_util_table_create": ([i32, vp, i32, vp, vp, p(vp)], C.c_int),
        "ca_util_table_destroy": ([vp], C.c_int),
        "ca_util_table_update": ([vp, vp, i32, vp, vp], C.c_int),
        "ca_util_table_set_added": ([vp, vp, vp, i32], C.c_int),
        "ca_util_calculate": ([vp, i32, i32, C.c_int64, vp, p(C.c_float)], C.c_int),
        "ca_util_device_results": ([vp, p(vp)], C.c_int),
        "ca_multi_create": ([p(vp), i32, p(vp)], C.c_int),
        "ca_multi_destroy": ([vp], C.c_int),
        "ca_multi_estimate_plan_create": ([vp, vp, vp, vp, vp, i32, p(vp)], C.c_int),
        "ca_multi_estimate_plan_run": ([vp, vp, p(i32), vp, vp, vp], C.c_int),
        "ca_multi_estimate_plan_stats": ([vp, p(i32), p(i32), vp, i32], C.c_int),
        "ca_multi_estimate_plan_rerun_units": ([vp, p(i32)], C.c_int),
        "ca_multi_estimate_plan_destroy": ([vp], C.c_int),
        "ca_multi_estimate_batch": ([vp, vp, vp, vp, vp, i32, vp, p(i32), vp, vp, vp], C.c_int),
        "ca_multi_removal_plan_create": ([vp, vp, i32, vp, vp, vp, vp, p(vp)], C.c_int),
        "ca_multi_removal_plan_run": ([vp, vp, i32, p(i32), vp, vp], C.c_int),
        "ca_multi_removal_plan_stats": ([vp, p(i32), p(i32), vp, i32], C.c_int),
        "ca_multi_removal_plan_rerun_units": ([vp, p(i32)], C.c_int),
        "ca_multi_removal_plan_timings": ([vp, vp, i32], C.c_int),
        "ca_multi_removal_plan_destroy": ([vp], C.c_int),
        "ca_multi_find_nodes_to_remove": ([vp, vp, i32, vp, vp, vp, vp, vp, i32, p(i32), vp, vp], C.c_int),
        "ca_plan_removals": ([vp, vp, i32, vp, vp, vp, vp, i32, vp, vp, i32, p(i32), vp, vp, i32, p(i32)], C.c_int),
        "ca_plan_last_moves": ([vp, vp, i32], C.c_int),
        "ca_plan_stats": ([vp, p(i32), p(i32), p(i32), p(C.c_float)], C.c_int),
        "ca_plan_last_path": ([vp], C.c_int),
        "ca_plan_chain_profile": ([vp, vp, i32, vp], C.c_int),
        "ca_interner_create": ([p(vp)], C.c_int),
        "ca_interner_destroy": ([vp], C.c_int),
        "ca_interner_size": ([vp, i32, p(i32), p(i32)], C.c_int),
        "ca_is_scalar_resource": ([C.c_char_p], C.c_int),
        "ca_intern_taint": ([vp, C.c_char_p, C.c_char_p, C.c_char_p, p(i32)], C.c_int),
        "ca_intern_label_pair": ([vp, C.c_char_p, C.c_char_p, p(i32)], C.c_int),
        "ca_intern_label_key": ([vp, C.c_char_p, p(i32)], C.c_int),
        "ca_intern_int_key": ([vp, C.c_char_p, p(i32)], C.c_int),
        "ca_intern_port": ([vp, C.c_char_p, C.c_char_p, i32, p(i32)], C.c_int),
        "ca_intern_resource": ([vp, C.c_char_p, p(i32)], C.c_int),
        "ca_intern_name": ([vp, C.c_char_p, p(i32)], C.c_int),
        "ca_intern_encode_node": ([vp, vp, i32, vp, i32, vp], C.c_int),
        "ca_intern_encode_tolerations": ([vp, vp, i32, vp, p(i32)], C.c_int),
        "ca_intern_encode_ports": ([vp, vp, i32, vp, p(i32)], C.c_int),
        "ca_intern_encode_node_selector": ([vp, vp, i32, vp, p(i32)], C.c_int),
        "ca_intern_compile_term": ([vp, vp, i32, vp, i32, p(i32), p(i32)], C.c_int),
    }
    for name, (args, res) in sigs.items():
        if path != LIB_PATH and not hasattr(lib, name):
            continue                      # an older diagnostics build (A/B runs)
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    _LIB = lib
    return lib


def _fast_copy(a: np.ndarray) -> np.ndarray:
    """Copy of a C-contiguous array through a byte view: numpy copies structured (record)
    arrays field by field (~100 us for 5 000 sweep results), bytes in one memcpy."""
    if a is None:
        return None
    return a.view(np.uint8).copy().view(a.dtype) if a.dtype.fields else a.copy()


def _check(status: int, what: str) -> None:
    if status != abi.CA_OK:
        raise CasimError(status, what)


def exported_symbols() -> list[str]:
    return [
        "ca_abi_version", "ca_abi_struct_sizes", "ca_device_count", "ca_status_string", "ca_host_alloc",
        "ca_host_free", "ca_mirror_create",
        "ca_mirror_destroy", "ca_mirror_clear", "ca_mirror_add_nodes", "ca_mirror_add_pods", "ca_mirror_remove_pod",
        "ca_mirror_remove_node", "ca_mirror_scope_blockers",
        "ca_mirror_fork", "ca_mirror_revert", "ca_mirror_commit", "ca_mirror_node_count", "ca_mirror_pod_node",
        "ca_mirror_node_pods", "ca_podset_create", "ca_podset_destroy", "ca_fits_any_node", "ca_check_predicates",
        "ca_fits_matrix", "ca_check_templates", "ca_expansion_plan_create", "ca_expansion_plan_run",
        "ca_expansion_plan_destroy", "ca_expansion_plan_kernel_ms", "ca_estimate_batch", "ca_estimate_plan_create", "ca_estimate_plan_run",
        "ca_estimate_plan_run_u16",
        "ca_estimate_plan_destroy", "ca_estimate_plan_stats", "ca_estimate_plan_chain_info", "ca_estimate_plan_rebase",
        "ca_estimate_plan_timings",
        "ca_estimate_plan_set_phase_timing",
        "ca_estimate_plan_group_ticks", "ca_estimate_plan_fetch", "ca_estimate_plan_device_results",
        "ca_go_sort_ranks",
        "ca_find_nodes_to_remove",
        "ca_removal_stats", "ca_removal_timings", "ca_removal_plan_create", "ca_removal_plan_run",
        "ca_removal_plan_destroy", "ca_removal_plan_sensitive_pods", "ca_removal_plan_phased",
        "ca_removal_plan_run_phase", "ca_sweep_compose", "ca_mirror_set_hints", "ca_mirror_get_hints",
        "ca_removal_candidate_ticks", "ca_filter_out_schedulable", "ca_filter_stats",
        "ca_util_table_create", "ca_util_table_destroy", "ca_util_calculate", "ca_util_device_results",
        "ca_util_table_update", "ca_util_table_set_added", "ca_multi_create", "ca_multi_destroy",
        "ca_multi_estimate_plan_create", "ca_multi_estimate_plan_run",
        "ca_multi_estimate_plan_stats", "ca_multi_estimate_plan_rerun_units", "ca_multi_estimate_plan_destroy", "ca_multi_estimate_batch",
        "ca_multi_removal_plan_create", "ca_multi_removal_plan_run", "ca_multi_removal_plan_stats",
        "ca_multi_removal_plan_rerun_units", "ca_multi_removal_plan_timings",
        "ca_multi_removal_plan_destroy", "ca_multi_find_nodes_to_remove",
        "ca_plan_removals", "ca_plan_last_moves", "ca_plan_stats", "ca_plan_last_path", "ca_plan_chain_profile",
        "ca_interner_create", "ca_interner_destroy", "ca_interner_size", "ca_is_scalar_resource", "ca_intern_taint",
        "ca_intern_label_pair", "ca_intern_label_key", "ca_intern_int_key", "ca_intern_port", "ca_intern_resource",
        "ca_intern_name", "ca_intern_encode_node", "ca_intern_encode_tolerations", "ca_intern_encode_ports",
        "ca_intern_encode_node_selector", "ca_intern_compile_term",
    ]


def go_sort_ranks(ranks, store: int = 0, limit: int = 0, device: int = 0) -> np.ndarray:
    """Go 1.19 sort.Slice of a slice by dense rank on the device (ca_go_sort_ranks): the
    permutation (perm[k] = input index of the element at position k)."""
    r = np.ascontiguousarray(ranks, dtype=np.uint32)
    perm = np.zeros(max(len(r), 1), np.int32)
    st = load().ca_go_sort_ranks(device, r.ctypes.data, len(r), store, limit, perm.ctypes.data)
    if st != abi.CA_OK:
        raise CasimError(st, "go_sort_ranks")
    return perm[: len(r)]


def sweep_compose(recs: np.ndarray, n_nodes: int, last_index: int) -> np.ndarray:
    """ca_sweep_compose: every block's exact input lastIndex from the blocks' MAP records
    (abi.CA_SWEEP_NOT_REACHED where the maps cannot carry the chain)."""
    r = np.ascontiguousarray(recs, dtype=abi.SWEEP_PHASE_DTYPE)
    lin = np.zeros(max(len(r), 1), np.int32)
    _check(load().ca_sweep_compose(r.ctypes.data, len(r), n_nodes, last_index, lin.ctypes.data, None),
           "ca_sweep_compose")
    return lin[: len(r)]


def device_count() -> int:
    n = C.c_int32(0)
    st = load().ca_device_count(C.byref(n))
    return n.value if st == abi.CA_OK else 0


@dataclass
class EstimateOutput:
    results: np.ndarray          # ESTIMATE_RESULT_DTYPE [G]
    sched_pod: np.ndarray        # int32 [total], CSR by group_off
    sched_node: np.ndarray       # int32 [total]
    last_index: int


@dataclass
class RemovalOutput:
    results: np.ndarray          # REMOVAL_RESULT_DTYPE [C]
    dest: np.ndarray             # int32 [M]
    hints: np.ndarray            # int32 [pods]
    last_index: int


@dataclass
class PlanOutput:
    results: np.ndarray          # PLAN_RESULT_DTYPE [C]
    moves: np.ndarray            # PLAN_MOVE_DTYPE [n_moves]
    hints: np.ndarray            # int32 [pods]
    last_index: int
    allowed: np.ndarray          # int32 [n_pdbs]: the PDB budgets after the call


@dataclass
class _PlanArgs:
    cand: np.ndarray
    mask: np.ndarray
    status: np.ndarray
    off: np.ndarray
    moves: np.ndarray
    hints: np.ndarray
    allowed: np.ndarray
    pdb_c: object
    keep: tuple
    res: np.ndarray
    out_moves: np.ndarray

    @property
    def pdb_ptr(self):
        return None if self.pdb_c is None else C.byref(self.pdb_c)

    def output(self, last_index: int, n_moves: int) -> PlanOutput:
        return PlanOutput(self.res, self.out_moves[:n_moves], self.hints, last_index, self.allowed)


def plan_args(candidates, dest_mask, cand_status, move_off, move_pods, hints, pdb_allowed=None, pdb_pod_off=None,
              pdb_pod=None) -> _PlanArgs:
    """Marshal the arguments of ca_plan_removals / or_plan_removals.  PDBs (optional):
    pdb_allowed[n_pdbs] DisruptionsAllowed, pdb_pod_off/pdb_pod the memberships (CSR by pod id)."""
    cand = np.ascontiguousarray(candidates, dtype=np.int32)
    status = np.ascontiguousarray(cand_status if cand_status is not None else np.zeros(len(cand)), dtype=np.int32)
    moves = np.ascontiguousarray(move_pods, dtype=np.int32)
    allowed = np.array(pdb_allowed if pdb_allowed is not None else [], dtype=np.int32)
    pdb_c, keep = None, ()
    if len(allowed):
        po = np.ascontiguousarray(pdb_pod_off, dtype=np.int32)
        pp = np.ascontiguousarray(pdb_pod if len(pdb_pod) else [0], dtype=np.int32)
        pdb_c = abi.PdbTableC(len(allowed), ptr(allowed), ptr(po), ptr(pp))
        keep = (po, pp)
    cap = 4 * len(moves) + 256
    return _PlanArgs(cand, np.ascontiguousarray(dest_mask, dtype=np.uint8), status,
                     np.ascontiguousarray(move_off, dtype=np.int32), moves,
                     np.array(hints, dtype=np.int32, copy=True), allowed, pdb_c, keep,
                     np.zeros(max(len(cand), 1), abi.PLAN_RESULT_DTYPE), np.zeros(cap, abi.PLAN_MOVE_DTYPE))


@dataclass
class FilterOutput:
    node: np.ndarray             # int32 [n]: node position per processed pod, -1 still pending
    pod_id: np.ndarray           # int32 [n]: mirror pod id of the added pod, -1
    hints: np.ndarray            # int32 [n]: hints after the call (Hints.Set)
    placed: int
    last_index: int
    evals: int
    n_overflowing: int


@dataclass
class _FilterArgs:
    order: np.ndarray
    n: int
    owner: object
    n_classes: int
    hints: np.ndarray
    node: np.ndarray
    pod_id: np.ndarray

    @property
    def owner_ptr(self):
        return None if self.owner is None else ptr(self.owner)

    def output(self, placed: int, last_index: int, evals: int, n_overflowing: int) -> FilterOutput:
        return FilterOutput(self.node[: self.n], self.pod_id[: self.n], self.hints[: self.n], placed, last_index,
                            evals, n_overflowing)


def filter_args(table: abi.PodTable, order=None, class_owner=None, hints=None) -> _FilterArgs:
    """Marshal the arguments of ca_filter_out_schedulable / or_filter_out_schedulable."""
    n_pods = len(table.pods)
    order = np.arange(n_pods, dtype=np.int32) if order is None else np.ascontiguousarray(order, dtype=np.int32)
    n = len(order)
    cls = table.pods["similar_class"]
    n_classes = int(cls.max()) + 1 if n_pods else 0
    owner = None
    if class_owner is not None:
        owner = np.full(max(n_classes, 1), -1, np.int32)
        co = np.ascontiguousarray(class_owner, dtype=np.int32)
        owner[: min(len(co), n_classes)] = co[:n_classes]
        n_classes = max(n_classes, 0)
    h = np.full(max(n, 1), -1, np.int32)
    if hints is not None:
        h[:n] = np.asarray(hints, dtype=np.int32)
    return _FilterArgs(order if n else np.zeros(1, np.int32), n, owner, max(n_classes, 0), h,
                       np.full(max(n, 1), -1, np.int32), np.full(max(n, 1), -1, np.int32))


class Mirror:
    """A ``ca_mirror``: the HBM-resident ClusterSnapshot data plane."""

    backend_name = "native"

    def __init__(self, device: int = 0):
        self.lib = load()
        h = C.c_void_p()
        _check(self.lib.ca_mirror_create(device, C.byref(h)), "ca_mirror_create")
        self.h = h
        self._keep: list = []

    def close(self) -> None:
        if self.h:
            self.lib.ca_mirror_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    # -- snapshot data plane --------------------------------------------------
    def clear(self) -> None:
        _check(self.lib.ca_mirror_clear(self.h), "ca_mirror_clear")

    def add_nodes(self, nodes: np.ndarray) -> int:
        nodes = np.ascontiguousarray(nodes, dtype=abi.NODE_DTYPE)
        first = C.c_int32(0)
        _check(self.lib.ca_mirror_add_nodes(self.h, ptr(nodes), len(nodes), C.byref(first)), "ca_mirror_add_nodes")
        return first.value

    def add_pods(self, table: abi.PodTable, idx, node_pos) -> np.ndarray:
        idx = np.ascontiguousarray(idx, dtype=np.int32)
        node_pos = np.ascontiguousarray(node_pos, dtype=np.int32)
        out = np.zeros(len(idx), np.int32)
        _check(self.lib.ca_mirror_add_pods(self.h, table.ref, ptr(idx), ptr(node_pos), len(idx), ptr(out)),
               "ca_mirror_add_pods")
        return out

    def remove_pod(self, pod_id: int) -> None:
        _check(self.lib.ca_mirror_remove_pod(self.h, pod_id), "ca_mirror_remove_pod")

    def remove_node(self, pos: int) -> None:
        _check(self.lib.ca_mirror_remove_node(self.h, pos), "ca_mirror_remove_node")

    def scope_blockers(self) -> int:
        n = C.c_int32(0)
        _check(self.lib.ca_mirror_scope_blockers(self.h, C.byref(n)), "ca_mirror_scope_blockers")
        return n.value

    def fork(self) -> None:
        _check(self.lib.ca_mirror_fork(self.h), "ca_mirror_fork")

    def revert(self) -> None:
        _check(self.lib.ca_mirror_revert(self.h), "ca_mirror_revert")

    def commit(self) -> None:
        _check(self.lib.ca_mirror_commit(self.h), "ca_mirror_commit")

    def node_count(self) -> int:
        n = C.c_int32(0)
        _check(self.lib.ca_mirror_node_count(self.h, C.byref(n)), "ca_mirror_node_count")
        return n.value

    def pod_node(self, pod_id: int) -> int:
        n = C.c_int32(0)
        _check(self.lib.ca_mirror_pod_node(self.h, pod_id, C.byref(n)), "ca_mirror_pod_node")
        return n.value

    def node_pods(self, node: int) -> list[int]:
        cap = 256
        while True:
            out = np.zeros(cap, np.int32)
            n = C.c_int32(0)
            st = self.lib.ca_mirror_node_pods(self.h, node, ptr(out), cap, C.byref(n))
            if st == abi.CA_ECAPACITY:
                cap = n.value
                continue
            _check(st, "ca_mirror_node_pods")
            return out[: n.value].tolist()

    # -- predicate checker ----------------------------------------------------
    def fits_any_node(self, table: abi.PodTable, pod: int, match=None, last_index: int = 0):
        ms, mask = abi.match_spec(*(match or ()))
        li = C.c_int32(last_index)
        out = C.c_int32(-1)
        pf = C.c_int32(0)
        ev = C.c_uint64(0)
        _check(self.lib.ca_fits_any_node(self.h, table.ref, pod, C.byref(ms), C.byref(li), C.byref(out),
                                         C.byref(pf), C.byref(ev)), "ca_fits_any_node")
        del mask
        return out.value, li.value, pf.value, ev.value

    def check_predicates(self, table: abi.PodTable, pod: int, node: int):
        r = abi.PredResultC()
        _check(self.lib.ca_check_predicates(self.h, table.ref, pod, node, C.byref(r)), "ca_check_predicates")
        return r.type, r.plugin, r.reasons, r.taint

    def podset(self, table: abi.PodTable) -> "PodSet":
        """`table` resident in device memory, for several calls (close() it after)."""
        return PodSet(self, table)

    def fits_matrix(self, table: abi.PodTable) -> np.ndarray:
        s = C.c_void_p()
        _check(self.lib.ca_podset_create(self.h, table.ref, C.byref(s)), "ca_podset_create")
        try:
            out = np.zeros((len(table), self.node_count()), np.uint8)
            _check(self.lib.ca_fits_matrix(self.h, s, ptr(out)), "ca_fits_matrix")
        finally:
            self.lib.ca_podset_destroy(s)
        return out

    # -- estimator ------------------------------------------------------------
    def estimate(self, table: abi.PodTable, group_off, pod_idx, templates: np.ndarray, max_nodes: int,
                 last_index: int = 0, want_nodes: bool = True, podset=None) -> EstimateOutput:
        with EstimatePlan(self, table, group_off, pod_idx, templates, podset=podset) as plan:
            return plan.run(max_nodes, last_index, want_nodes=want_nodes)

    def check_templates(self, table: abi.PodTable, samples, templates: np.ndarray, podset=None,
                        verdict_only: bool = False, out=None) -> np.ndarray:
        """ComputeExpansionOption's feasibility (orchestrator.go:455-481) for every (node
        group, pod equivalence group): [G][E] ca_pred_result of CheckPredicates(sample pod,
        a fresh copy of the template), or with verdict_only a [G][E] uint8 (1 = fits).
        `podset`: a resident PodSet of `table` (else the table is uploaded for the call);
        `out`: a caller buffer of the result shape (e.g. page-locked)."""
        sm = np.ascontiguousarray(samples, dtype=np.int32)
        tm = np.ascontiguousarray(templates, dtype=abi.TEMPLATE_DTYPE)
        if out is None:
            out = np.zeros((len(tm), len(sm)), np.uint8 if verdict_only else abi.PRED_RESULT_DTYPE)
        own = podset is None
        ps = PodSet(self, table) if own else podset
        try:
            full, ok = (None, out) if verdict_only else (out, None)
            _check(self.lib.ca_check_templates(self.h, ps.h, ptr(sm), len(sm), ptr(tm), len(tm),
                                               ptr(full) if full is not None else None,
                                               ptr(ok) if ok is not None else None),
                   "ca_check_templates")
        finally:
            if own:
                ps.close()
        return out

    # -- removal simulator ----------------------------------------------------
    def filter_out_schedulable(self, table: abi.PodTable, order=None, class_owner=None, hints=None,
                               last_index: int = 0, podset=None) -> FilterOutput:
        """ca_filter_out_schedulable: TrySchedulePods(pending, ScheduleAnywhere, breakOnFailure=false)
        committed into the mirror (filter_out_schedulable.go:95-124)."""
        a = filter_args(table, order, class_owner, hints)
        li = C.c_int32(last_index)
        ev = C.c_uint64(0)
        ov = C.c_int32(0)
        placed = C.c_int32(0)
        _check(self.lib.ca_filter_out_schedulable(self.h, table.ref, podset.h if podset is not None else None,
                                                  ptr(a.order), a.n, a.owner_ptr, a.n_classes, ptr(a.hints),
                                                  C.byref(li), ptr(a.node), ptr(a.pod_id), C.byref(ov),
                                                  C.byref(ev), C.byref(placed)), "ca_filter_out_schedulable")
        return a.output(placed.value, li.value, ev.value, ov.value)

    def filter_stats(self) -> dict:
        out = (C.c_float * 16)()
        self.lib.ca_filter_stats(self.h, out, 16)
        return {"kernel_ms": out[0], "total_ms": out[1], "phases": int(out[2]), "block_steps": int(out[3]),
                "ring_scans": int(out[4]), "windows": int(out[5]), "seq_share": out[6],
                "walk_cycles_per_pod": out[7], "path": "bitmap" if out[8] else "window", "shapes": int(out[9]),
                "static_classes": int(out[10]), "fb_cycles_per_pod": [out[11], out[12], out[13]],
                "static_in_lds": bool(out[15])}

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
        _check(self.lib.ca_find_nodes_to_remove(self.h, ptr(cand), len(cand), ptr(mask), ptr(status), ptr(off),
                                                ptr(moves), ptr(hints), C.byref(li), ptr(res), ptr(dest)),
               "ca_find_nodes_to_remove")
        return RemovalOutput(res, dest[: len(moves)], hints, li.value)

    def plan_removals(self, candidates, dest_mask, cand_status, move_off, move_pods, hints, last_index: int = 0,
                      max_removable: int = 0, pdb_allowed=None, pdb_pod_off=None, pdb_pod=None) -> PlanOutput:
        """ca_plan_removals: Planner.categorizeNodes' loop with canPersist=true; commits into
        the mirror.  hints: per mirror pod (len = the mirror's pod count)."""
        a = plan_args(candidates, dest_mask, cand_status, move_off, move_pods, hints, pdb_allowed, pdb_pod_off, pdb_pod)
        li = C.c_int32(last_index)
        nm = C.c_int32(0)
        _check(self.lib.ca_plan_removals(self.h, ptr(a.cand), len(a.cand), ptr(a.mask), ptr(a.status), ptr(a.off),
                                         ptr(a.moves), int(max_removable), a.pdb_ptr, ptr(a.hints), len(a.hints),
                                         C.byref(li), ptr(a.res), ptr(a.out_moves), len(a.out_moves), C.byref(nm)),
               "ca_plan_removals")
        if nm.value > len(a.out_moves):
            a.out_moves = np.zeros(nm.value, abi.PLAN_MOVE_DTYPE)
            self.lib.ca_plan_last_moves(self.h, ptr(a.out_moves), nm.value)
        a.res = a.res[: len(a.cand)]
        return a.output(li.value, nm.value)

    def plan_stats(self) -> dict:
        r, c, s = C.c_int32(0), C.c_int32(0), C.c_int32(0)
        t = C.c_float(0)
        _check(self.lib.ca_plan_stats(self.h, C.byref(r), C.byref(c), C.byref(s), C.byref(t)), "ca_plan_stats")
        return {"rounds": r.value, "conflicts": c.value, "simulated": s.value, "total_ms": t.value,
                "path": "chain" if self.lib.ca_plan_last_path(self.h) == 1 else "speculative"}

    def plan_chain_profile(self) -> dict:
        """Phase cycle counters and host timings of the last device-chain planner call."""
        cyc = np.zeros(32, np.uint64)
        hm = np.zeros(5, np.float32)
        k = self.lib.ca_plan_chain_profile(self.h, cyc.ctypes.data, 32, hm.ctypes.data)
        names = ["init", "lists", "pdb", "fork", "hint", "scan", "add", "commit", "revert", "total", "blocks",
                 "windows", "handoffs", "bulk", "prep", "win", "loadchk", "skyb", "r_pod", "r_win", "r_blk", "r_sky",
                 "r_add", "r_npods", "r_nblk", "r_nwin", "r_nsky", "r_nruns"]
        out = {nm: int(v) for nm, v in zip(names, cyc[:max(k, 0)])}
        out.update({h: float(v) for h, v in zip(["sync_ms", "launch_kernel_ms", "kernel_ms", "readback_ms",
                                                   "replay_ms"], hm)})
        return out

    def set_hints(self, hints) -> None:
        """The mirror's resident HintingSimulator hints (node per mirror pod, -1 = none)."""
        h = np.ascontiguousarray(hints, dtype=np.int32)
        _check(self.lib.ca_mirror_set_hints(self.h, ptr(h), len(h)), "ca_mirror_set_hints")

    def get_hints(self, n_pods: int) -> np.ndarray:
        h = np.zeros(n_pods, np.int32)
        _check(self.lib.ca_mirror_get_hints(self.h, ptr(h), n_pods), "ca_mirror_get_hints")
        return h

    def candidate_ticks(self, n_candidates: int) -> np.ndarray:
        """Per candidate of the last sweep: device time of its simulation, us."""
        a = np.zeros(n_candidates, np.uint64)
        _check(self.lib.ca_removal_candidate_ticks(self.h, a.ctypes.data_as(C.POINTER(C.c_uint64)), n_candidates),
               "ca_removal_candidate_ticks")
        return a.astype(np.float64) / 100.0

    def removal_stats(self) -> dict:
        r, k, t = C.c_int32(0), C.c_float(0), C.c_float(0)
        self.lib.ca_removal_stats(self.h, C.byref(r), C.byref(k), C.byref(t))
        tm = (C.c_float * 4)()
        self.lib.ca_removal_timings(self.h, tm, 4)
        return {"rounds": r.value, "kernel_ms": k.value, "total_ms": t.value, "exact_ms": float(tm[1]),
                "walk_ms": float(tm[2])}


class RemovalPlan:
    """``ca_removal_plan``: FindNodesToRemove inputs resident in HBM for repeated sweeps."""

    def __init__(self, mirror: Mirror, candidates, dest_mask, cand_status, move_off, move_pods):
        self.m = mirror
        self.lib = mirror.lib
        self.cand = np.ascontiguousarray(candidates, dtype=np.int32)
        mask = np.ascontiguousarray(dest_mask, dtype=np.uint8)
        status = np.ascontiguousarray(cand_status if cand_status is not None else np.zeros(len(self.cand)),
                                      dtype=np.int32)
        off = np.ascontiguousarray(move_off, dtype=np.int32)
        self.moves = np.ascontiguousarray(move_pods, dtype=np.int32)
        p = C.c_void_p()
        _check(self.lib.ca_removal_plan_create(mirror.h, ptr(self.cand), len(self.cand), ptr(mask), ptr(status),
                                               ptr(off), ptr(self.moves), C.byref(p)), "ca_removal_plan_create")
        self.h = p
        self.results = np.zeros(len(self.cand), abi.REMOVAL_RESULT_DTYPE)
        self._dest = PinnedArray(self.lib, max(len(self.moves), 1), np.int32)

    def run(self, last_index: int = 0, hints=None, want_dest: bool = False) -> RemovalOutput:
        """One sweep.  hints=None: the mirror's resident hints are used and updated
        (Mirror.set_hints / get_hints); else a per-pod array, updated in place."""
        h = None if hints is None else np.ascontiguousarray(hints, dtype=np.int32)
        li = C.c_int32(last_index)
        dest = self._dest.array if want_dest else None
        _check(self.lib.ca_removal_plan_run(self.h, ptr(h) if h is not None else None, C.byref(li), ptr(self.results),
                                            ptr(dest) if dest is not None else None), "ca_removal_plan_run")
        return RemovalOutput(_fast_copy(self.results), dest[: len(self.moves)].copy() if dest is not None else None, h,
                             li.value)

    # -- the phased sweep of one block (casim.h "one process per GPU"; shard.sweep_sharded) --
    def sensitive_pods(self) -> int:
        v = C.c_int64(0)
        _check(self.lib.ca_removal_plan_sensitive_pods(self.h, C.byref(v)), "ca_removal_plan_sensitive_pods")
        return v.value

    def phased(self) -> bool:
        v = C.c_int32(0)
        _check(self.lib.ca_removal_plan_phased(self.h, C.byref(v)), "ca_removal_plan_phased")
        return bool(v.value)

    def run_phase(self, rec: np.ndarray, hints: np.ndarray, last_index: int, want_dest: bool = True):
        """One phase (rec["kind"]) of this block; rec is a 1-element SWEEP_PHASE_DTYPE array,
        updated in place; hints (int32, per mirror pod) read, and for RESOLVE updated for the
        block's pods.  RESOLVE returns the block's RemovalOutput (dest: the block's moves)."""
        assert rec.dtype == abi.SWEEP_PHASE_DTYPE and rec.flags["C_CONTIGUOUS"]
        assert hints.dtype == np.int32 and hints.flags["C_CONTIGUOUS"]
        li = C.c_int32(last_index)
        dest = self._dest.array if want_dest else None
        _check(self.lib.ca_removal_plan_run_phase(self.h, rec.ctypes.data, ptr(hints), C.byref(li), ptr(self.results),
                                                  ptr(dest) if dest is not None else None), "ca_removal_plan_run_phase")
        if int(rec["kind"][0]) != abi.CA_SWEEP_PHASE_RESOLVE:
            return None
        return RemovalOutput(_fast_copy(self.results), dest[: len(self.moves)].copy() if dest is not None else None,
                             hints, li.value)

    def close(self) -> None:
        if self.h:
            self.lib.ca_removal_plan_destroy(self.h)
            self.h = None
            self._dest.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class PinnedArray:
    """A numpy array over ca_host_alloc (page-locked) memory."""

    def __init__(self, lib, n: int, dtype):
        self.lib = lib
        dt = np.dtype(dtype)
        p = C.c_void_p()
        _check(lib.ca_host_alloc(max(n, 1) * dt.itemsize, C.byref(p)), "ca_host_alloc")
        self.p = p
        buf = (C.c_char * (max(n, 1) * dt.itemsize)).from_address(p.value)
        self.array = np.frombuffer(buf, dtype=dt, count=n)

    def close(self) -> None:
        if self.p:
            self.array = None
            self.lib.ca_host_free(self.p)
            self.p = None


class PinnedRows:
    """Reusable page-locked (ca_host_alloc) arrays for rows a caller builds and uploads
    every loop: the H2D copy then runs at the link's DMA rate instead of through a
    pageable staging copy."""

    def __init__(self, lib=None):
        self.lib = lib or load()
        self._bufs = {}

    def zeros(self, key: str, n: int, dtype, zero: bool = True) -> np.ndarray:
        dt = np.dtype(dtype)
        b = self._bufs.get(key)
        if b is None or b.array.size < n or b.array.dtype != dt:
            if b is not None:
                b.close()
            b = PinnedArray(self.lib, max(n, 1), dt)
            self._bufs[key] = b
        a = b.array[:n]
        if zero:
            a.view(np.uint8)[...] = 0
        return a

    def close(self) -> None:
        for b in self._bufs.values():
            b.close()
        self._bufs = {}


class PodSet:
    """A pod table resident in device memory (ca_podset): uploaded once, reused by calls."""

    def __init__(self, mirror: "Mirror", table: abi.PodTable):
        self.lib = mirror.lib
        self.table = table                      # keeps the host arrays alive
        h = C.c_void_p()
        _check(self.lib.ca_podset_create(mirror.h, table.ref, C.byref(h)), "ca_podset_create")
        self.h = h

    def close(self) -> None:
        if self.h:
            self.lib.ca_podset_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class EstimatePlan:
    """``ca_estimate_plan``: device-resident groups for repeated Estimate batches."""

    def __init__(self, mirror: Mirror, table: abi.PodTable, group_off, pod_idx, templates: np.ndarray,
                 podset: "PodSet" = None):
        """`podset`: a resident PodSet of `table` to use (else the table is uploaded here)."""
        self.m = mirror
        self.lib = mirror.lib
        self.group_off = np.ascontiguousarray(group_off, dtype=np.int32)
        self.pod_idx = np.ascontiguousarray(pod_idx, dtype=np.int32)
        self.templates = np.ascontiguousarray(templates, dtype=abi.TEMPLATE_DTYPE)
        self.G = len(self.templates)
        self.total = int(self.group_off[-1]) if len(self.group_off) else 0
        if podset is None:
            s = C.c_void_p()
            _check(self.lib.ca_podset_create(mirror.h, table.ref, C.byref(s)), "ca_podset_create")
            self.podset = s
        else:
            self.podset = None
            s = podset.h
        p = C.c_void_p()
        st = self.lib.ca_estimate_plan_create(mirror.h, s, ptr(self.group_off), ptr(self.pod_idx),
                                              ptr(self.templates), self.G, C.byref(p))
        if st != abi.CA_OK:
            if self.podset:
                self.lib.ca_podset_destroy(self.podset)
            raise CasimError(st, "ca_estimate_plan_create")
        self.h = p
        n = max(self.total, 1)
        self._pinned = PinnedArray(self.lib, 2 * n, np.int32)     # sched_pod | sched_node
        self.sched_pod = self._pinned.array[:n]
        self.sched_node = self._pinned.array[n:]
        self.results = np.zeros(self.G, abi.ESTIMATE_RESULT_DTYPE)
        self._pinned16 = None

    def run_u16(self, max_nodes: int, last_index: int = 0, copy: bool = True) -> EstimateOutput:
        """One Estimate batch with the scheduled pods as 16-bit podset indices
        (ca_estimate_plan_run_u16: podsets of at most 65535 pods; 0xFFFF = not scheduled).
        sched_node of the returned output is None."""
        if self._pinned16 is None:
            self._pinned16 = PinnedArray(self.lib, max(self.total, 1), np.uint16)
            # the call's arguments, built once (a step of the bench's headline loop is ~0.5 ms:
            # the per-call ctypes conversions were a few percent of it)
            self._u16_lim = abi.LimiterC(0, 0)
            self._u16_li = C.c_int32(0)
            self._u16_args = (self.h, C.byref(self._u16_lim), C.byref(self._u16_li), ptr(self.results),
                              ptr(self._pinned16.array))
            self._u16_view = self._pinned16.array[: self.total]
        self._u16_lim.max_nodes = max_nodes
        self._u16_li.value = last_index
        _check(self.lib.ca_estimate_plan_run_u16(*self._u16_args), "ca_estimate_plan_run_u16")
        if copy:
            return EstimateOutput(_fast_copy(self.results), self._u16_view.copy(), None, self._u16_li.value)
        return EstimateOutput(self.results, self._u16_view, None, self._u16_li.value)

    def run(self, max_nodes: int, last_index: int = 0, want_nodes: bool = True, copy: bool = True,
            device_results: bool = False) -> EstimateOutput:
        """One Estimate batch.  With copy=False the returned arrays are views of the plan's
        page-locked result buffers, overwritten by the next run.  With device_results=True
        the scheduled pods stay in device memory (sched_pod/sched_node of the returned
        output are None; fetch() copies them)."""
        lim = abi.LimiterC(max_nodes, 0)
        li = C.c_int32(last_index)
        if device_results:
            _check(self.lib.ca_estimate_plan_run(self.h, C.byref(lim), C.byref(li), ptr(self.results), None, None),
                   "ca_estimate_plan_run")
            return EstimateOutput(_fast_copy(self.results) if copy else self.results, None, None, li.value)
        _check(self.lib.ca_estimate_plan_run(self.h, C.byref(lim), C.byref(li), ptr(self.results),
                                             ptr(self.sched_pod), ptr(self.sched_node) if want_nodes else None),
               "ca_estimate_plan_run")
        f = _fast_copy if copy else (lambda a: a)
        return EstimateOutput(f(self.results), f(self.sched_pod[: self.total]), f(self.sched_node[: self.total]),
                              li.value)

    def fetch(self) -> np.ndarray:
        """The scheduled pods of the last run, copied from device memory."""
        out = np.full(max(self.total, 1), -1, np.int32)
        _check(self.lib.ca_estimate_plan_fetch(self.h, ptr(out)), "ca_estimate_plan_fetch")
        return out[: self.total]

    def stats(self) -> dict:
        r, a, b, c = C.c_int32(0), C.c_float(0), C.c_float(0), C.c_float(0)
        self.lib.ca_estimate_plan_stats(self.h, C.byref(r), C.byref(a), C.byref(b), C.byref(c))
        sens, succ = C.c_int32(0), C.c_int32(0)
        self.lib.ca_estimate_plan_chain_info(self.h, C.byref(sens), C.byref(succ))
        t = (C.c_float * 9)()
        self.lib.ca_estimate_plan_timings(self.h, t, 9)
        names = ("score_ms", "merge_ms", "emit_ms", "chain_ms", "compact_ms", "d2h_ms", "host_ms")
        return {"rounds": r.value, "chain_ms": a.value, "sort_ms": b.value, "total_ms": c.value,
                "lin_sensitive": sens.value, "had_success": succ.value,
                "phases": {k: float(v) for k, v in zip(names, t)},
                "results_path": ("copied", "published", "publisher_gave_up")[int(t[7])],
                "decoupled": bool(t[8])}

    def set_phase_timing(self, on: bool) -> None:
        """Per-phase timing events on later runs (on by default; off keeps them off the
        launch path — stats() phases then read 0)."""
        _check(self.lib.ca_estimate_plan_set_phase_timing(self.h, 1 if on else 0), "ca_estimate_plan_set_phase_timing")

    def chain_info(self) -> tuple:
        """(lastIndex-sensitive, had a FitsAnyNode success) of the last run: one call."""
        sens, succ = C.c_int32(0), C.c_int32(0)
        self.lib.ca_estimate_plan_chain_info(self.h, C.byref(sens), C.byref(succ))
        return sens.value, succ.value

    def rebase(self, results: np.ndarray, last_index_in: int) -> int:
        """ca_estimate_plan_rebase: `results` (this plan's last run, a writable copy) re-based
        in place to the exact input lastIndex; returns the batch's exact output."""
        lo = C.c_int32(0)
        _check(self.lib.ca_estimate_plan_rebase(self.h, ptr(results), last_index_in, C.byref(lo)),
               "ca_estimate_plan_rebase")
        return lo.value

    def group_ticks(self) -> np.ndarray:
        """Per group of the last run: (chain device time in us, single-pod steps)."""
        n = self.lib.ca_estimate_plan_group_ticks(self.h, None, 0)
        a = np.zeros(max(n, 0), np.uint64)
        if n > 0:
            self.lib.ca_estimate_plan_group_ticks(self.h, a.ctypes.data_as(C.POINTER(C.c_uint64)), n)
        return np.stack([(a & 0xFFFFFFFF).astype(np.float64) / 100.0, (a >> 32).astype(np.float64)], axis=1)

    def close(self) -> None:
        if self.h:
            self.lib.ca_estimate_plan_destroy(self.h)
            if self.podset:
                self.lib.ca_podset_destroy(self.podset)
            self.h = None
            self.sched_pod = self.sched_node = None
            self._pinned.close()
            if self._pinned16 is not None:
                self._pinned16.close()
                self._pinned16 = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class ExpansionPlan:
    """ComputeExpansionOption's check with the node groups resident (ca_expansion_plan_*,
    include/casim.h; CA/core/scaleup/orchestrator/orchestrator.go:455-481): the templates'
    test-node rows are uploaded once; run() checks a pod set's samples against all of them."""

    def __init__(self, mirror: "Mirror", templates: np.ndarray):
        self.lib = load()
        self.mirror = mirror
        self.templates = np.ascontiguousarray(templates, dtype=abi.TEMPLATE_DTYPE)
        h = C.c_void_p()
        _check(self.lib.ca_expansion_plan_create(mirror.h, ptr(self.templates), len(self.templates), C.byref(h)),
               "ca_expansion_plan_create")
        self.h = h

    def run(self, podset: "PodSet", samples, verdict_only: bool = False, out=None) -> np.ndarray:
        """[G][E] ca_pred_result (or with verdict_only a [G][E] uint8, 1 = fits), as
        Mirror.check_templates returns it."""
        sm = np.ascontiguousarray(samples, dtype=np.int32)
        G = len(self.templates)
        if out is None:
            out = np.zeros((G, len(sm)), np.uint8 if verdict_only else abi.PRED_RESULT_DTYPE)
        full, ok = (None, out) if verdict_only else (out, None)
        _check(self.lib.ca_expansion_plan_run(self.h, podset.h, ptr(sm), len(sm),
                                              ptr(full) if full is not None else None,
                                              ptr(ok) if ok is not None else None), "ca_expansion_plan_run")
        return out

    @property
    def kernel_ms(self) -> float:
        """The last run's kernel time (HIP events)."""
        v = C.c_float(0)
        _check(self.lib.ca_expansion_plan_kernel_ms(self.h, C.byref(v)), "ca_expansion_plan_kernel_ms")
        return v.value

    def close(self) -> None:
        if self.h:
            self.lib.ca_expansion_plan_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class UtilTable:
    """Device-resident node/pod table for utilization.Calculate over every node
    (include/casim.h ca_util_*; CA/simulator/utilization/info.go:48-127)."""

    def __init__(self, device: int, nodes: np.ndarray, pod_off: np.ndarray, pods: np.ndarray):
        self.lib = load()
        self.nodes = np.ascontiguousarray(nodes, abi.UTIL_NODE_DTYPE)
        self.pod_off = np.ascontiguousarray(pod_off, np.int32)
        self.pods = np.ascontiguousarray(pods, abi.UTIL_POD_DTYPE)
        if len(self.pod_off) != len(self.nodes) + 1 or int(self.pod_off[-1]) != len(self.pods):
            raise ValueError("pod_off must have n_nodes + 1 entries ending at len(pods)")
        h = C.c_void_p()
        _check(self.lib.ca_util_table_create(device, ptr(self.nodes), len(self.nodes), ptr(self.pod_off),
                                             ptr(self.pods), C.byref(h)), "ca_util_table_create")
        self.h = h
        self.kernel_ms = 0.0

    def update(self, nodes: np.ndarray, pod_off: np.ndarray, pods: np.ndarray) -> None:
        """New rows (the snapshot changed), in the table's device buffers."""
        self.nodes = np.ascontiguousarray(nodes, abi.UTIL_NODE_DTYPE)
        self.pod_off = np.ascontiguousarray(pod_off, np.int32)
        self.pods = np.ascontiguousarray(pods, abi.UTIL_POD_DTYPE)
        _check(self.lib.ca_util_table_update(self.h, ptr(self.nodes), len(self.nodes), ptr(self.pod_off),
                                             ptr(self.pods)), "ca_util_table_update")

    def set_added(self, node, pods) -> None:
        """Pods added to the snapshot since the rows were set: pods[k] on node[k]."""
        self.added_node = np.ascontiguousarray(node, np.int32)
        self.added_pods = np.ascontiguousarray(pods, abi.UTIL_POD_DTYPE)
        _check(self.lib.ca_util_table_set_added(self.h, ptr(self.added_node), ptr(self.added_pods),
                                                len(self.added_node)), "ca_util_table_set_added")

    def calculate(self, skip_daemonset_pods: bool, skip_mirror_pods: bool, now_ns: int,
                  to_host: bool = True, out: np.ndarray = None):
        """out: a caller's (page-locked) result array, else a new one."""
        if to_host and out is None:
            out = np.zeros(len(self.nodes), abi.UTIL_INFO_DTYPE)
        ms = C.c_float(0)
        _check(self.lib.ca_util_calculate(self.h, int(skip_daemonset_pods), int(skip_mirror_pods), int(now_ns),
                                          ptr(out) if to_host else None, C.byref(ms)), "ca_util_calculate")
        self.kernel_ms = ms.value
        return out

    def close(self) -> None:
        if self.h:
            self.lib.ca_util_table_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Multi:
    """``ca_multi``: replicated mirrors, one per device.  The caller keeps
    them identical; `mirrors` may repeat a device (tests shard over two mirrors on one GPU)."""

    def __init__(self, mirrors):
        self.mirrors = list(mirrors)
        self.lib = self.mirrors[0].lib
        arr = (C.c_void_p * len(self.mirrors))(*[m.h for m in self.mirrors])
        h = C.c_void_p()
        _check(self.lib.ca_multi_create(arr, len(self.mirrors), C.byref(h)), "ca_multi_create")
        self.h = h

    def for_each(self, fn):
        """Apply a snapshot change to every replica, in order."""
        return [fn(m) for m in self.mirrors]

    def close(self) -> None:
        if self.h:
            self.lib.ca_multi_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class MultiEstimatePlan:
    """``ca_multi_estimate_plan``: node groups in contiguous blocks over the replicas."""

    def __init__(self, multi: Multi, table: abi.PodTable, group_off, pod_idx, templates: np.ndarray):
        self.lib = multi.lib
        self.group_off = np.ascontiguousarray(group_off, dtype=np.int32)
        self.pod_idx = np.ascontiguousarray(pod_idx, dtype=np.int32)
        self.templates = np.ascontiguousarray(templates, dtype=abi.TEMPLATE_DTYPE)
        self.G = len(self.templates)
        self.total = int(self.group_off[-1]) if len(self.group_off) else 0
        h = C.c_void_p()
        _check(self.lib.ca_multi_estimate_plan_create(multi.h, table.ref, ptr(self.group_off), ptr(self.pod_idx),
                                                      ptr(self.templates), self.G, C.byref(h)),
               "ca_multi_estimate_plan_create")
        self.h = h
        n = max(self.total, 1)
        self._pinned = PinnedArray(self.lib, 2 * n, np.int32)
        self.sched_pod = self._pinned.array[:n]
        self.sched_node = self._pinned.array[n:]
        self.results = np.zeros(self.G, abi.ESTIMATE_RESULT_DTYPE)

    def run(self, max_nodes: int, last_index: int = 0, want_nodes: bool = True, copy: bool = True) -> EstimateOutput:
        lim = abi.LimiterC(max_nodes, 0)
        li = C.c_int32(last_index)
        _check(self.lib.ca_multi_estimate_plan_run(self.h, C.byref(lim), C.byref(li), ptr(self.results),
                                                   ptr(self.sched_pod), ptr(self.sched_node) if want_nodes else None),
               "ca_multi_estimate_plan_run")
        f = _fast_copy if copy else (lambda a: a)
        return EstimateOutput(f(self.results), f(self.sched_pod[: self.total]), f(self.sched_node[: self.total]),
                              li.value)

    def stats(self) -> dict:
        nb, rr = C.c_int32(0), C.c_int32(0)
        first = np.zeros(65, np.int32)
        self.lib.ca_multi_estimate_plan_stats(self.h, C.byref(nb), C.byref(rr), ptr(first), len(first))
        ru = C.c_int32(0)
        self.lib.ca_multi_estimate_plan_rerun_units(self.h, C.byref(ru))
        return {"blocks": nb.value, "reruns": rr.value, "block_first_group": first[: nb.value + 1].tolist(),
                "rerun_groups": ru.value}

    def close(self) -> None:
        if self.h:
            self.lib.ca_multi_estimate_plan_destroy(self.h)
            self.h = None
            self._pinned.close()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class MultiRemovalPlan:
    """``ca_multi_removal_plan``: FindNodesToRemove candidates in contiguous blocks."""

    def __init__(self, multi: Multi, candidates, dest_mask, cand_status, move_off, move_pods):
        self.lib = multi.lib
        self.cand = np.ascontiguousarray(candidates, dtype=np.int32)
        mask = np.ascontiguousarray(dest_mask, dtype=np.uint8)
        status = np.ascontiguousarray(cand_status if cand_status is not None else np.zeros(len(self.cand)),
                                      dtype=np.int32)
        off = np.ascontiguousarray(move_off, dtype=np.int32)
        self.moves = np.ascontiguousarray(move_pods, dtype=np.int32)
        h = C.c_void_p()
        _check(self.lib.ca_multi_removal_plan_create(multi.h, ptr(self.cand), len(self.cand), ptr(mask), ptr(status),
                                                     ptr(off), ptr(self.moves), C.byref(h)),
               "ca_multi_removal_plan_create")
        self.h = h
        self.results = np.zeros(len(self.cand), abi.REMOVAL_RESULT_DTYPE)

    def run(self, hints, last_index: int = 0) -> RemovalOutput:
        hints = np.array(hints, dtype=np.int32, copy=True)
        dest = np.full(max(len(self.moves), 1), -1, np.int32)
        li = C.c_int32(last_index)
        _check(self.lib.ca_multi_removal_plan_run(self.h, ptr(hints), len(hints), C.byref(li), ptr(self.results),
                                                  ptr(dest)), "ca_multi_removal_plan_run")
        return RemovalOutput(_fast_copy(self.results), dest[: len(self.moves)], hints, li.value)

    def stats(self) -> dict:
        nb, rr = C.c_int32(0), C.c_int32(0)
        first = np.zeros(65, np.int32)
        self.lib.ca_multi_removal_plan_stats(self.h, C.byref(nb), C.byref(rr), ptr(first), len(first))
        ru = C.c_int32(0)
        self.lib.ca_multi_removal_plan_rerun_units(self.h, C.byref(ru))
        tm = np.zeros(5, np.float32)
        self.lib.ca_multi_removal_plan_timings(self.h, tm.ctypes.data, 5)
        return {"blocks": nb.value, "reruns": rr.value, "block_first_candidate": first[: nb.value + 1].tolist(),
                "rerun_candidates": ru.value,
                "phase_ms": dict(zip(("probe", "map", "compose", "resolve", "fixup"), tm.tolist()))}

    def close(self) -> None:
        if self.h:
            self.lib.ca_multi_removal_plan_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


# ---- interning through the C ABI (casim.h "interning"; host-only, no device needed) ------

class _StrPair(C.Structure):
    _fields_ = [("key", C.c_char_p), ("value", C.c_char_p)]


class _TaintStr(C.Structure):
    _fields_ = [("key", C.c_char_p), ("value", C.c_char_p), ("effect", C.c_char_p)]


class _TolerationStr(C.Structure):
    _fields_ = [("key", C.c_char_p), ("op", C.c_char_p), ("value", C.c_char_p), ("effect", C.c_char_p)]


class _PortStr(C.Structure):
    _fields_ = [("host_ip", C.c_char_p), ("protocol", C.c_char_p), ("host_port", C.c_int32), ("reserved", C.c_int32)]


class _RequirementStr(C.Structure):
    _fields_ = [("key", C.c_char_p), ("op", C.c_char_p), ("values", C.POINTER(C.c_char_p)), ("n_values", C.c_int32),
                ("is_field", C.c_int32)]


def _b(x) -> bytes:
    return (x or "").encode()


class CInterner:
    """``ca_interner``: the library's interning (what a cgo shim binds), driven with Python
    strings.  Ids and encodings equal autoscaler_amd/intern.py's (tests/test_intern_c.py)."""

    def __init__(self):
        self.lib = load()
        h = C.c_void_p()
        _check(self.lib.ca_interner_create(C.byref(h)), "ca_interner_create")
        self.h = h

    def close(self):
        if self.h:
            self.lib.ca_interner_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _id(self, fn, *a) -> int:
        i = C.c_int32(0)
        _check(getattr(self.lib, fn)(self.h, *a, C.byref(i)), fn)
        return i.value

    def taint(self, k, v, e):
        return self._id("ca_intern_taint", _b(k), _b(v), _b(e))

    def label_pair(self, k, v):
        return self._id("ca_intern_label_pair", _b(k), _b(v))

    def label_key(self, k):
        return self._id("ca_intern_label_key", _b(k))

    def int_key(self, k):
        return self._id("ca_intern_int_key", _b(k))

    def port(self, ip, proto, port):
        return self._id("ca_intern_port", _b(ip), _b(proto), int(port))

    def resource(self, name):
        return self._id("ca_intern_resource", _b(name))

    def name(self, n):
        return self._id("ca_intern_name", _b(n))

    def size(self, universe: int) -> tuple:
        n, o = C.c_int32(0), C.c_int32(0)
        _check(self.lib.ca_interner_size(self.h, universe, C.byref(n), C.byref(o)), "ca_interner_size")
        return n.value, o.value

    def encode_node(self, labels: dict, taints, rec) -> None:
        """labels {k: v}; taints [(key, value, effect)]; rec: an abi.NODE_DTYPE record (array of 1)."""
        lb = (_StrPair * max(len(labels), 1))(*[_StrPair(_b(k), _b(v)) for k, v in labels.items()])
        tt = (_TaintStr * max(len(taints), 1))(*[_TaintStr(_b(k), _b(v), _b(e)) for k, v, e in taints])
        _check(self.lib.ca_intern_encode_node(self.h, lb, len(labels), tt, len(taints), rec.ctypes.data),
               "ca_intern_encode_node")

    def encode_tolerations(self, tols, rec) -> int:
        """tols [(key, op, value, effect)]; rec: abi.POD_DTYPE array of 1.  Returns out_of_scope."""
        tt = (_TolerationStr * max(len(tols), 1))(*[_TolerationStr(_b(k), _b(o), _b(v), _b(e)) for k, o, v, e in tols])
        o = C.c_int32(0)
        _check(self.lib.ca_intern_encode_tolerations(self.h, tt, len(tols), rec.ctypes.data, C.byref(o)),
               "ca_intern_encode_tolerations")
        return o.value

    def encode_ports(self, ports, rec) -> int:
        """ports [(host_ip, protocol, host_port)] of the pod's containers."""
        pp = (_PortStr * max(len(ports), 1))(*[_PortStr(_b(i), _b(pr), int(pt), 0) for i, pr, pt in ports])
        o = C.c_int32(0)
        _check(self.lib.ca_intern_encode_ports(self.h, pp, len(ports), rec.ctypes.data, C.byref(o)),
               "ca_intern_encode_ports")
        return o.value

    def encode_node_selector(self, sel: dict, rec) -> int:
        ss = (_StrPair * max(len(sel), 1))(*[_StrPair(_b(k), _b(v)) for k, v in sel.items()])
        o = C.c_int32(0)
        _check(self.lib.ca_intern_encode_node_selector(self.h, ss, len(sel), rec.ctypes.data, C.byref(o)),
               "ca_intern_encode_node_selector")
        return o.value

    def compile_term(self, reqs) -> tuple:
        """reqs [(key, op, [values], is_field)] -> (abi.REQ_DTYPE rows, out_of_scope)."""
        keep = []
        rr = (_RequirementStr * max(len(reqs), 1))()
        for i, (k, op, vals, f) in enumerate(reqs):
            va = (C.c_char_p * max(len(vals), 1))(*[_b(v) for v in vals])
            keep.append(va)
            rr[i] = _RequirementStr(_b(k), _b(op), C.cast(va, C.POINTER(C.c_char_p)), len(vals), int(bool(f)))
        out = np.zeros(max(len(reqs), 1), abi.REQ_DTYPE)
        nr, o = C.c_int32(0), C.c_int32(0)
        _check(self.lib.ca_intern_compile_term(self.h, rr, len(reqs), out.ctypes.data, len(out), C.byref(nr),
                                               C.byref(o)), "ca_intern_compile_term")
        del keep
        return out[: nr.value], o.value
