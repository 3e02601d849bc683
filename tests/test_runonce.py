"""RunOnce's simulation legs end to end (autoscaler_amd/runonce.py): FilterOutSchedulable
-> expansion options -> Estimate -> utilization / empty nodes -> FindNodesToRemove, on the
CPU restatement (host glue, CPU) and on the HIP mirror against it (GPU), step by step."""
import numpy as np
import pytest

from autoscaler_amd import runonce


def _oracle_run(w):
    import pyoracle
    from autoscaler_amd import workloads as W
    o = pyoracle.OracleState()
    W.load_filter(o, w.filt)
    return runonce.run(o, pyoracle.runonce_cpu_util, w)


def test_runonce_small_oracle(oracle_lib):
    w = runonce.c5_runonce(n_nodes=600, n_pending=1500, n_groups=12)
    r = _oracle_run(w)
    s = r.sizes
    assert 0 < s["placed_by_filter"] < s["pending"]
    assert s["sweep_candidates"] > 0 and s["pods_to_move"] > 0
    assert s["estimate_items"] > 0
    assert (r.est_results["status"] == 0).all()
    # the candidates are exactly the nodes below the threshold, in node order
    assert np.all(np.diff(r.candidates) > 0)
    assert (r.util["utilization"][r.candidates] < runonce.UTIL_THRESHOLD).all()


@pytest.mark.gpu
@pytest.mark.parametrize("size", ["small", "c5"])
def test_runonce_gpu_parity(size, oracle_lib):
    from autoscaler_amd import native
    from autoscaler_amd import workloads as W
    w = runonce.c5_runonce() if size == "c5" else runonce.c5_runonce(n_nodes=2000, n_pending=4000, n_groups=30)
    ro = _oracle_run(w)
    m = native.Mirror(0)
    W.load_filter(m, w.filt)

    util = runonce.DeviceUtil(0)
    expand = runonce.DeviceExpansion()
    rg = runonce.run(m, util, w, expand_fn=expand)
    # the resident plan's results against the one-shot call's (full reason records)
    ps = m.podset(w.filt.pending)
    samples = np.array([g[0] for g in runonce._equivalence_groups(
        w.filt.pending.pods, w.filt.order[rg.filter_node < 0])], np.int32)
    ok = expand(m, ps, samples, w.templates)                # the loop's verdict-only form
    full = expand.plan.run(ps, samples)                     # the same plan, full records
    assert full.tobytes() == m.check_templates(w.filt.pending, samples, w.templates, podset=ps).tobytes()
    assert ok.dtype == np.uint8 and np.array_equal(ok, (full["type"] == 0).astype(np.uint8))
    ps.close()
    expand.close()
    # the full rows through one table, as a second form of the same step
    fullu = runonce.UtilInput(w, rg.filter_node, "full")
    t = native.UtilTable(0, fullu.nodes, fullu.off, fullu.pods)
    assert t.calculate(False, False, w.now_ns).tobytes() == rg.util.tobytes()
    t.close()
    util.close()
    m.close()
    eq = runonce.compare(ro, rg)
    assert all(eq.values()), eq
    assert ro.last_index == rg.last_index
