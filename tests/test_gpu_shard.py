"""One process per GPU (shard.py over torch.distributed): the C3 sweep in the three phases of
casim.h "one process per GPU" (PROBE, MAP, ca_sweep_compose, RESOLVE, one all-gather of the
560-B records per phase) and the node-group chain of Estimate with re-basing, every rank
on its own mirror replica.  The box has one GPU, so the ranks share device 0 and exchange
over gloo (the bench's N > 1 run uses RCCL over xGMI, one device per rank); the protocol,
plans and kernels are the same.  Results must equal the oracle's sequential call bit for bit
 on every rank, hints included, over two loops."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _paths():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "oracle"), os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _sweep_worker(rank, world, port, n_nodes, q):
    _paths()
    import torch.distributed as dist
    import pyoracle
    from autoscaler_amd import native, shard
    from autoscaler_amd import workloads as W

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = W.c3(n_nodes=n_nodes)
        blocks = shard.split_blocks(np.diff(w.move_off), world)
        a, b = blocks[rank], blocks[rank + 1]
        m = native.Mirror(0)
        W.load_sweep(m, w)
        plan = native.RemovalPlan(m, w.candidates[a:b], w.dest_mask, w.cand_status[a:b],
                                  (w.move_off[a:b + 1] - w.move_off[a]).astype(np.int32),
                                  w.move_pods[w.move_off[a]:w.move_off[b]])
        ex = shard.Exchange(shard.torch_gather_bytes(dist, "cpu"))
        sb, ph = shard.sweep_setup(plan, ex, rank, a == b)
        o = pyoracle.OracleState()
        W.load_sweep(o, w)
        ok, notes = True, []
        hints = np.full(len(w.table), -1, np.int32)
        h_ref = hints.copy()
        L = 7
        for loop in range(3):                     # fresh, hinted, hinted again
            res, dest, final_L, st = shard.sweep_sharded(plan, L, hints, len(w.nodes), ex, rank, blocks, w.move_off,
                                                         w.move_pods, sb, ph)
            ref = o.find_nodes_to_remove(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods, h_ref, L)
            good = (np.array_equal(res, ref.results) and np.array_equal(dest, ref.dest)
                    and final_L == ref.last_index and np.array_equal(hints, ref.hints))
            ok &= bool(good)
            notes.append((loop, bool(good), st["reached"], st["serial_blocks"]))
            h_ref, L = ref.hints.copy(), ref.last_index
        plan.close()
        m.close()
        q.put((rank, bool(ok), notes))
    finally:
        dist.destroy_process_group()


def _estimate_worker(rank, world, port, seed, q):
    _paths()
    import torch.distributed as dist
    import pyoracle
    from autoscaler_amd import native, shard
    from estgen import _encode_estimate, _estimate_inputs

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng, nodes, pods, templates, groups = _estimate_inputs(seed, n_groups=9, n_pods=70)
        table, node_recs, tm, off, pod_idx = _encode_estimate(nodes, pods, templates, groups)
        max_nodes = [0, 1, 3, 40][seed % 4]
        L0 = [0, 3, 11][seed % 3]
        blocks = shard.split_blocks(np.diff(off), world)
        a, b = blocks[rank], blocks[rank + 1]
        m = native.Mirror(0)
        if len(node_recs):
            m.add_nodes(node_recs)
        plan = native.EstimatePlan(m, table, (off[a:b + 1] - off[a]).astype(np.int32), pod_idx[off[a]:off[b]], tm[a:b])
        ex = shard.Exchange(shard.torch_gather_bytes(dist, "cpu"))
        res, sched, final_L, reruns = shard.estimate_sharded(plan, max_nodes, L0, ex, rank, blocks, off)
        o = pyoracle.OracleState()
        o.clear()
        if len(node_recs):
            o.add_nodes(node_recs)
        ro = o.estimate(table, off, pod_idx, tm, max_nodes, L0)
        ok = np.array_equal(res, ro.results) and final_L == ro.last_index
        for g in range(len(tm)):
            if int(ro.results[g]["status"]) != 0:
                continue
            s, n = off[g], int(ro.results[g]["n_scheduled"])
            ok &= np.array_equal(sched[s:s + n], ro.sched_pod[s:s + n])
        plan.close()
        m.close()
        q.put((rank, bool(ok), reruns))
    finally:
        dist.destroy_process_group()


def _spawn(target, world, *args):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return sorted(res, key=lambda r: r[0])


@pytest.mark.parametrize("world,n_nodes", [(2, 300), (3, 1500), (4, 5000)])
def test_sharded_sweep_phases(world, n_nodes):
    res = _spawn(_sweep_worker, world, n_nodes)
    assert all(ok for _, ok, _ in res), res
    # full C3: the fresh loop's blocks compose (no block runs a whole call after its
    # predecessor), as test_multi_sweep_c3_full asserts for the library's form
    for _, _, notes in res:
        print(notes)
        if n_nodes >= 5000:
            assert notes[0][3] == 0, notes


@pytest.mark.parametrize("seed", range(4))
def test_sharded_estimate_rebase(seed):
    res = _spawn(_estimate_worker, 3, seed)
    assert all(ok for _, ok, _ in res), res


def _cut_worker(rank, world, port, n_nodes, q):
    """An out-of-scope pod to move in a middle block: every plan runs whole calls (the
    phases need every block free of a prefix-protocol cut), the cut candidate reports
    OUT_OF_SCOPE and every later one NOT_RUN, as one mirror's call does."""
    _paths()
    import dataclasses
    import torch.distributed as dist
    from autoscaler_amd import abi, native, shard
    from autoscaler_amd import workloads as W

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = W.c3(n_nodes=n_nodes)
        pods = w.table.pods.copy()
        c_mid = len(w.candidates) // 2
        pods["flags"][int(w.move_pods[w.move_off[c_mid]])] |= abi.CA_POD_OUT_OF_SCOPE
        w = dataclasses.replace(w, table=abi.PodTable(pods))
        blocks = shard.split_blocks(np.diff(w.move_off), world)
        a, b = blocks[rank], blocks[rank + 1]
        m = native.Mirror(0)
        W.load_sweep(m, w)
        ref = m.find_nodes_to_remove(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods,
                                     np.full(len(w.table), -1, np.int32), 5)
        plan = native.RemovalPlan(m, w.candidates[a:b], w.dest_mask, w.cand_status[a:b],
                                  (w.move_off[a:b + 1] - w.move_off[a]).astype(np.int32),
                                  w.move_pods[w.move_off[a]:w.move_off[b]])
        ex = shard.Exchange(shard.torch_gather_bytes(dist, "cpu"))
        sb, ph = shard.sweep_setup(plan, ex, rank, a == b)
        hints = np.full(len(w.table), -1, np.int32)
        res, dest, L, st = shard.sweep_sharded(plan, 5, hints, len(w.nodes), ex, rank, blocks, w.move_off, w.move_pods,
                                               sb, ph)
        ok = np.array_equal(res, ref.results) and np.array_equal(dest, ref.dest) and L == ref.last_index
        ok &= np.array_equal(hints, ref.hints)
        ok &= int(res[c_mid]["reason"]) == abi.CA_UNREMOVABLE_OUT_OF_SCOPE
        ok &= bool((res["reason"][c_mid + 1:] == abi.CA_UNREMOVABLE_NOT_RUN).all())
        ok &= st["serial_blocks"] == world
        plan.close()
        m.close()
        q.put((rank, bool(ok), st))
    finally:
        dist.destroy_process_group()


def test_sharded_sweep_prefix_cut():
    res = _spawn(_cut_worker, 3, 600)
    assert all(ok for _, ok, _ in res), res
