"""FilterOutSchedulable on the HIP path (ca_filter_out_schedulable, filter.hip) vs the CPU
restatement (or_filter_out_schedulable): bit-exact node per pod, mirror pod ids, hints,
lastIndex, evaluation count and overflowing controllers; then the state both leave
behind is compared through a second call."""
import numpy as np
import pytest

from autoscaler_amd import native
from autoscaler_amd import workloads as W
from test_filter_out import run_both

pytestmark = pytest.mark.gpu


def _eq(rg, ro, what=""):
    assert rg.placed == ro.placed, what
    assert np.array_equal(rg.node, ro.node), (what, np.nonzero(rg.node != ro.node)[0][:10])
    assert np.array_equal(rg.pod_id, ro.pod_id), what
    assert np.array_equal(rg.hints, ro.hints), what
    assert (rg.last_index, rg.evals, rg.n_overflowing) == (ro.last_index, ro.evals, ro.n_overflowing), what


@pytest.mark.parametrize("seed", range(16))
def test_filter_api_random(seed, oracle_lib):
    """Processor facade over the GPU mirror == over the oracle (statuses, hints, L, evals)."""
    _, ref = run_both(oracle_lib.OracleState, seed, last_index=seed % 7)
    _, got = run_both(lambda: native.Mirror(0), seed, last_index=seed % 7)
    assert got == ref


@pytest.mark.parametrize("n_nodes,n_pending", [(10, 300), (64, 2000), (700, 3000)])
def test_filter_api_random_sizes(n_nodes, n_pending, oracle_lib):
    _, ref = run_both(oracle_lib.OracleState, 99, n_nodes=n_nodes, n_pending=n_pending)
    _, got = run_both(lambda: native.Mirror(0), 99, n_nodes=n_nodes, n_pending=n_pending)
    assert got == ref


CONFIGS = {
    "small": dict(n_nodes=500, pods_per_node=20, n_pending=2000),
    "tight": dict(n_nodes=800, pods_per_node=20, n_pending=6000, util_low=(0.9, 0.97), util_high=(0.97, 1.0)),
    "loose": dict(n_nodes=2000, pods_per_node=20, n_pending=6000, util_low=(0.2, 0.4), util_high=(0.5, 0.7)),
    # mixed runs: scanning and hinted pods placed together, windows that wrap the ring,
    # a ring shorter than the 64-node window, a cluster that fills up on the way
    "loose-hinted": dict(n_nodes=1500, pods_per_node=20, n_pending=6000, hint_frac=0.6,
                         util_low=(0.1, 0.3), util_high=(0.3, 0.6)),
    "loose-tiny": dict(n_nodes=37, pods_per_node=10, n_pending=900, hint_frac=0.3,
                       util_low=(0.1, 0.3), util_high=(0.3, 0.5)),
    "loose-filling": dict(n_nodes=300, pods_per_node=20, n_pending=6000, hint_frac=0.4,
                          util_low=(0.3, 0.5), util_high=(0.5, 0.7)),
    "nohints": dict(n_nodes=3000, pods_per_node=20, n_pending=8000, hint_frac=0.0),
    "allhints": dict(n_nodes=3000, pods_per_node=20, n_pending=8000, hint_frac=1.0),
    "full": dict(),
}


@pytest.mark.parametrize("path", ["bitmap", "window"])
@pytest.mark.parametrize("taints", [False, True], ids=["resources", "c4"])
@pytest.mark.parametrize("cfg", list(CONFIGS))
def test_filter_c5(cfg, taints, path, oracle_lib, monkeypatch):
    """Both kernels: the feasibility-bitmap walk (every C5 pod qualifies) and the window
    sequencer (forced with CASIM_FO_WINDOW)."""
    if path == "window":
        monkeypatch.setenv("CASIM_FO_WINDOW", "1")
    w = W.c5_filter(taints=taints, **CONFIGS[cfg])
    g, o = native.Mirror(0), oracle_lib.OracleState()
    W.load_filter(g, w)
    W.load_filter(o, w)
    rg = g.filter_out_schedulable(w.pending, w.order, w.class_owner, w.hints, 3)
    assert g.filter_stats()["path"] == path
    ro = o.filter_out_schedulable(w.pending, w.order, w.class_owner, w.hints, 3)
    _eq(rg, ro, cfg)
    # the state left behind: a second pass of everything (hints from the first) matches,
    # and the pods still pending stay pending (idempotence)
    rg2 = g.filter_out_schedulable(w.pending, w.order, w.class_owner, rg.hints, rg.last_index)
    ro2 = o.filter_out_schedulable(w.pending, w.order, w.class_owner, ro.hints, ro.last_index)
    _eq(rg2, ro2, cfg + " second pass")
    left = w.order[rg.node < 0]
    r3 = g.filter_out_schedulable(w.pending, left, w.class_owner, None, rg.last_index)
    assert r3.placed == 0
    g.close()


@pytest.mark.parametrize("n_nodes,n_pending", [(1000, 3000), (4000, 12000)])
def test_filter_fork_revert(n_nodes, n_pending, oracle_lib):
    """Placements land on the current fork level: Revert drops them (delta.go).  The larger
    case applies its placements to the host rows on several threads (add_placed_batch)."""
    w = W.c5_filter(n_nodes=n_nodes, pods_per_node=20, n_pending=n_pending)
    g, o = native.Mirror(0), oracle_lib.OracleState()
    for b in (g, o):
        W.load_filter(b, w)
        b.fork()
    rg = g.filter_out_schedulable(w.pending, w.order, w.class_owner, w.hints, 0)
    ro = o.filter_out_schedulable(w.pending, w.order, w.class_owner, w.hints, 0)
    _eq(rg, ro, "forked")
    g.revert()
    o.revert()
    rg = g.filter_out_schedulable(w.pending, w.order, w.class_owner, None, 0)
    ro = o.filter_out_schedulable(w.pending, w.order, w.class_owner, None, 0)
    _eq(rg, ro, "after revert")
    g.close()


def test_filter_no_class_owner_and_empty(oracle_lib):
    w = W.c5_filter(n_nodes=300, pods_per_node=20, n_pending=1500)
    g, o = native.Mirror(0), oracle_lib.OracleState()
    W.load_filter(g, w)
    W.load_filter(o, w)
    e = g.filter_out_schedulable(w.pending, np.zeros(0, np.int32), None, None, 5)
    assert e.placed == 0 and e.last_index == 5
    rg = g.filter_out_schedulable(w.pending, None, None, None, 7)
    ro = o.filter_out_schedulable(w.pending, None, None, None, 7)
    _eq(rg, ro, "table order, no cap")
    g.close()


def test_filter_dead_shapes(oracle_lib):
    """Pending pods whose shape fits no node (RunOnce's backlog): their shapes share one
    all-zero dyn row, so the call stays on the bitmap walk with > 64 distinct shapes."""
    from autoscaler_amd import runonce
    w = runonce.c5_runonce(n_nodes=3000, n_pending=6000, n_groups=4).filt
    g, o = native.Mirror(0), oracle_lib.OracleState()
    W.load_filter(g, w)
    W.load_filter(o, w)
    rg = g.filter_out_schedulable(w.pending, w.order, w.class_owner, w.hints, 3)
    st = g.filter_stats()
    assert st["path"] == "bitmap", st
    ro = o.filter_out_schedulable(w.pending, w.order, w.class_owner, w.hints, 3)
    _eq(rg, ro, "dead shapes")
    g.close()
