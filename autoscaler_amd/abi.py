"""ctypes / numpy mirror of ``include/casim.h``.

The numpy structured dtypes below are the single Python-side definition of the
ABI records; ``ctypes`` structures are derived for by-reference arguments.  A
binding test checks every size against ``ca_abi_struct_sizes`` exported by the
library, so a drift between this file and the header fails loudly.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

CASIM_ABI_VERSION = 3

# status codes
CA_OK, CA_EINVAL, CA_ENOTFOUND, CA_EEXISTS, CA_EDEVICE, CA_ECAPACITY, CA_EUNSUPPORTED, CA_ESTATE, CA_ENOTRUN = range(9)

CA_MAX_SCALAR = 8
CA_LABEL_WORDS = 4
CA_PORT_WORDS = 2
CA_MAX_INT_KEYS = 4

CA_NODE_UNSCHEDULABLE = 0x1
CA_NODE_ANTI_AFFINITY_PODS = 0x2

CA_POD_HAS_SCALAR_KEYS = 0x001
CA_POD_HAS_NONTPU_SCALAR_KEYS = 0x002
CA_POD_TOLERATES_UNSCHED = 0x004
CA_POD_AFFINITY_FILTER = 0x008
CA_POD_PREFILTER_FAIL = 0x010
CA_POD_PREFILTER_NAMES = 0x020
CA_POD_DAEMONSET = 0x040
CA_POD_HOSTNAME_DEPENDENT = 0x080
CA_POD_OUT_OF_SCOPE = 0x100
CA_POD_REQUIRED_ANTI_AFFINITY = 0x200

CA_OP_IN, CA_OP_NOTIN, CA_OP_EXISTS, CA_OP_DOESNOTEXIST, CA_OP_GT, CA_OP_LT, CA_OP_FIELD_EQ, CA_OP_FIELD_NE, \
    CA_OP_FALSE = range(1, 10)

CA_PLUGIN_NONE = 0
CA_PLUGIN_NODE_UNSCHEDULABLE = 1
CA_PLUGIN_NODE_NAME = 2
CA_PLUGIN_TAINT_TOLERATION = 3
CA_PLUGIN_NODE_AFFINITY = 4
CA_PLUGIN_NODE_PORTS = 5
CA_PLUGIN_NODE_RESOURCES_FIT = 6

PLUGIN_NAMES = {
    CA_PLUGIN_NODE_UNSCHEDULABLE: "NodeUnschedulable",
    CA_PLUGIN_NODE_NAME: "NodeName",
    CA_PLUGIN_TAINT_TOLERATION: "TaintToleration",
    CA_PLUGIN_NODE_AFFINITY: "NodeAffinity",
    CA_PLUGIN_NODE_PORTS: "NodePorts",
    CA_PLUGIN_NODE_RESOURCES_FIT: "NodeResourcesFit",
}

CA_PRED_OK, CA_PRED_NOT_SCHEDULABLE, CA_PRED_INTERNAL, CA_PRED_UNSUPPORTED = 0, 1, 2, 3

CA_REASON_TOO_MANY_PODS = 0x1
CA_REASON_INSUFF_CPU = 0x2
CA_REASON_INSUFF_MEMORY = 0x4
CA_REASON_INSUFF_EPHEMERAL = 0x8
CA_REASON_INSUFF_SCALAR0 = 0x100

CA_MATCH_ALL, CA_MATCH_RANGE, CA_MATCH_MASK = 0, 1, 2

CA_UNREMOVABLE_NONE = 0
CA_UNREMOVABLE_NO_PLACE = 12
CA_UNREMOVABLE_BLOCKED_BY_POD = 13
CA_UNREMOVABLE_UNEXPECTED_ERROR = 14
CA_UNREMOVABLE_OUT_OF_SCOPE = 100
CA_UNREMOVABLE_NOT_RUN = 101

# --------------------------------------------------------------------------
# record dtypes (C layout: align=True)
# --------------------------------------------------------------------------
NODE_DTYPE = np.dtype([
    ("alloc_milli_cpu", "<i8"), ("alloc_memory", "<i8"), ("alloc_ephemeral", "<i8"), ("alloc_pods", "<i8"),
    ("alloc_scalar", "<i8", (CA_MAX_SCALAR,)),
    ("taints", "<u8"),
    ("label_pairs", "<u8", (CA_LABEL_WORDS,)),
    ("label_keys", "<u8"),
    ("int_label", "<i8", (CA_MAX_INT_KEYS,)),
    ("int_label_valid", "<u4"), ("flags", "<u4"), ("name_id", "<i4"), ("reserved", "<i4"),
], align=True)

POD_DTYPE = np.dtype([
    ("req_milli_cpu", "<i8"), ("req_memory", "<i8"), ("req_ephemeral", "<i8"),
    ("req_scalar", "<i8", (CA_MAX_SCALAR,)),
    ("score_milli_cpu", "<i8"), ("score_memory", "<i8"),
    ("tolerated_taints", "<u8"),
    ("port_conflict", "<u8", (CA_PORT_WORDS,)),
    ("port_use", "<u8", (CA_PORT_WORDS,)),
    ("node_selector", "<u8", (CA_LABEL_WORDS,)),
    ("aff_term_first", "<i4"), ("aff_term_count", "<i4"),
    ("prefilter_first", "<i4"), ("prefilter_count", "<i4"),
    ("node_name_id", "<i4"), ("flags", "<u4"), ("similar_class", "<i4"), ("tpu_scalar_mask", "<u4"),
], align=True)

REQ_DTYPE = np.dtype([("op", "<i4"), ("key", "<i4"), ("bound", "<i8"), ("pairs", "<u8", (CA_LABEL_WORDS,))],
                     align=True)
TERM_DTYPE = np.dtype([("first", "<i4"), ("count", "<i4")], align=True)

TEMPLATE_DTYPE = np.dtype([
    ("node", NODE_DTYPE),
    ("used_milli_cpu", "<i8"), ("used_memory", "<i8"), ("used_ephemeral", "<i8"),
    ("used_scalar", "<i8", (CA_MAX_SCALAR,)),
    ("used_pods", "<i8"),
    ("used_ports", "<u8", (CA_PORT_WORDS,)),
], align=True)

ESTIMATE_RESULT_DTYPE = np.dtype([
    ("node_count", "<i4"), ("n_scheduled", "<i4"), ("nodes_added", "<i4"), ("last_index_in", "<i4"),
    ("last_index_out", "<i4"), ("status", "<i4"), ("evals", "<u8"),
], align=True)

REMOVAL_RESULT_DTYPE = np.dtype([
    ("removable", "<i4"), ("reason", "<i4"), ("n_placed", "<i4"), ("last_index_in", "<i4"), ("evals", "<u8"),
], align=True)

# planner (include/casim.h ca_plan_*)
PLAN_RESULT_DTYPE = np.dtype([
    ("removable", "<i4"), ("reason", "<i4"), ("n_placed", "<i4"), ("last_index_in", "<i4"), ("evals", "<u8"),
    ("first_move", "<i4"), ("n_moves", "<i4"), ("blocking_pod", "<i4"), ("risky", "<i4"),
], align=True)
PLAN_MOVE_DTYPE = np.dtype([("candidate", "<i4"), ("pod", "<i4"), ("new_pod", "<i4"), ("node", "<i4")])

# scale-down eligibility (include/casim.h ca_util_*)
CA_UTIL_CPU, CA_UTIL_MEM, CA_UTIL_GPU = 0, 1, 2
CA_UNODE_HAS_CPU, CA_UNODE_HAS_MEM, CA_UNODE_HAS_GPU, CA_UNODE_GPU_CONFIG = 0x1, 0x2, 0x4, 0x8
CA_UPOD_DAEMONSET, CA_UPOD_MIRROR, CA_UPOD_DELETED, CA_UPOD_MOVABLE, CA_UPOD_BLOCKING = 0x01, 0x02, 0x04, 0x08, 0x10
CA_UTIL_OK, CA_UTIL_NO_CPU, CA_UTIL_ZERO_CPU, CA_UTIL_NO_MEM, CA_UTIL_ZERO_MEM = 0, 1, 2, 3, 4

UTIL_NODE_DTYPE = np.dtype([("alloc_milli", "<i8", (3,)), ("flags", "<u4"), ("_pad", "<u4")], align=True)
UTIL_POD_DTYPE = np.dtype([
    ("req_milli", "<i8", (3,)), ("deletion_ns", "<i8"), ("grace_s", "<i8"), ("flags", "<u4"), ("_pad", "<u4"),
], align=True)
UTIL_INFO_DTYPE = np.dtype([
    ("cpu", "<f8"), ("mem", "<f8"), ("gpu", "<f8"), ("utilization", "<f8"), ("resource", "<i4"),
    ("status", "<i4"), ("empty", "<i4"), ("_pad", "<i4"),
], align=True)


class PodTableC(C.Structure):
    _fields_ = [
        ("pods", C.c_void_p), ("n_pods", C.c_int32), ("n_terms", C.c_int32),
        ("terms", C.c_void_p), ("reqs", C.c_void_p), ("n_reqs", C.c_int32),
        ("n_prefilter_names", C.c_int32), ("prefilter_names", C.c_void_p),
    ]


class MatchSpecC(C.Structure):
    _fields_ = [("kind", C.c_int32), ("lo", C.c_int32), ("hi", C.c_int32), ("exclude", C.c_int32),
                ("mask", C.c_void_p)]


class PredResultC(C.Structure):
    _fields_ = [("type", C.c_int32), ("plugin", C.c_int32), ("reasons", C.c_uint32), ("taint", C.c_int32)]


PRED_RESULT_DTYPE = np.dtype([("type", np.int32), ("plugin", np.int32), ("reasons", np.uint32), ("taint", np.int32)])


class LimiterC(C.Structure):
    _fields_ = [("max_nodes", C.c_int32), ("reserved", C.c_int32)]


class PdbTableC(C.Structure):
    _fields_ = [("n_pdbs", C.c_int32), ("allowed", C.c_void_p), ("pod_off", C.c_void_p), ("pod_pdb", C.c_void_p)]


# ca_sweep_phase: one block's record of the phased sweep (casim.h "one process per GPU")
CA_SWEEP_PHASE_PROBE, CA_SWEEP_PHASE_MAP, CA_SWEEP_PHASE_RESOLVE = 1, 2, 3
CA_SWEEP_MAP_INTS = 130
CA_SWEEP_NOT_REACHED = -(2 ** 31)
SWEEP_PHASE_DTYPE = np.dtype([("kind", np.int32), ("est_base", np.int32), ("guess_base", np.int64), ("adv", np.int64),
                              ("succ", np.int32), ("n_sensitive", np.int32), ("map_ran", np.int32),
                              ("map_ok", np.int32), ("map", np.int32, (CA_SWEEP_MAP_INTS,))])

# sizes in ca_abi_struct_sizes order
EXPECTED_SIZES = [
    NODE_DTYPE.itemsize, POD_DTYPE.itemsize, REQ_DTYPE.itemsize, TERM_DTYPE.itemsize,
    C.sizeof(PodTableC), C.sizeof(MatchSpecC), C.sizeof(PredResultC), TEMPLATE_DTYPE.itemsize,
    C.sizeof(LimiterC), ESTIMATE_RESULT_DTYPE.itemsize, REMOVAL_RESULT_DTYPE.itemsize,
    UTIL_NODE_DTYPE.itemsize, UTIL_POD_DTYPE.itemsize, UTIL_INFO_DTYPE.itemsize,
    PLAN_RESULT_DTYPE.itemsize, PLAN_MOVE_DTYPE.itemsize, SWEEP_PHASE_DTYPE.itemsize,
    16, 24, 32, 24, 32,          # ca_str_pair, ca_taint_str, ca_toleration_str, ca_port_str, ca_requirement_str
]


def ptr(a: np.ndarray | None) -> int | None:
    """Address of a C-contiguous numpy array (None for None / empty)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"], "ABI arrays must be C-contiguous"
    return a.ctypes.data if a.size else None


class PodTable:
    """Owns the numpy arrays behind one ``ca_pod_table``."""

    def __init__(self, pods: np.ndarray, terms: np.ndarray | None = None, reqs: np.ndarray | None = None,
                 names: np.ndarray | None = None):
        self.pods = np.ascontiguousarray(pods, dtype=POD_DTYPE)
        self.terms = np.ascontiguousarray(terms if terms is not None else np.zeros(0, TERM_DTYPE), dtype=TERM_DTYPE)
        self.reqs = np.ascontiguousarray(reqs if reqs is not None else np.zeros(0, REQ_DTYPE), dtype=REQ_DTYPE)
        self.names = np.ascontiguousarray(names if names is not None else np.zeros(0, np.int32), dtype=np.int32)
        self.c = PodTableC(ptr(self.pods), len(self.pods), len(self.terms), ptr(self.terms), ptr(self.reqs),
                           len(self.reqs), len(self.names), ptr(self.names))

    def __len__(self) -> int:
        return len(self.pods)

    @property
    def ref(self):
        return C.byref(self.c)


def empty_pods(n: int) -> np.ndarray:
    p = np.zeros(n, POD_DTYPE)
    p["aff_term_count"] = -1
    p["node_name_id"] = -1
    p["similar_class"] = -1
    return p


def empty_nodes(n: int) -> np.ndarray:
    return np.zeros(n, NODE_DTYPE)


def match_spec(kind: int = CA_MATCH_ALL, lo: int = 0, hi: int = 0, exclude: int = -1,
               mask: np.ndarray | None = None) -> tuple[MatchSpecC, np.ndarray | None]:
    m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
    return MatchSpecC(kind, lo, hi, exclude, ptr(m)), m
