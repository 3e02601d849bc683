"""Multi-rank node-group sharding (autoscaler_amd/shard.py) over torch.distributed gloo,
world_size 2, on CPU.  Each rank runs its contiguous block of node groups from the
caller's lastIndex and the ranks fix up the lastIndex chain with one all_gather per
round; the union of the ranks' results must equal one sequential Estimate over every
group (the reference calls Estimate group after group with one shared checker,
CA/core/scaleup/orchestrator/orchestrator.go:487-488).  The per-block Estimate here is
the CPU restatement (test infrastructure), so the protocol is exercised without a GPU."""
import os
import socket

import numpy as np
import pytest

from autoscaler_amd.shard import run_sharded, walk


def test_walk_accepts_and_flags():
    # rank 1 ran from 0 but rank 0 moved lastIndex to 5 and rank 1 is sensitive
    assert walk([[0, 5, 1, 1], [0, 9, 1, 1]], 0) == (1, 5)
    # insensitive blocks are accepted whatever their input
    assert walk([[0, 5, 1, 1], [0, 9, 0, 1]], 0) == (-1, 9)
    # a block without a FitsAnyNode success passes lastIndex through
    assert walk([[3, 3, 0, 0], [3, 7, 1, 1]], 3) == (-1, 7)


def test_run_sharded_single_process_protocol():
    """Two simulated ranks driven in lockstep: rank 1 must re-run from rank 0's output."""
    calls = {0: [], 1: []}

    def make_run(r):
        def run(lin):
            calls[r].append(lin)
            return f"out{r}@{lin}", lin + 10 * (r + 1), 1, 1
        return run

    # lockstep all_gather for two "ranks" inside one process
    import threading
    barrier = threading.Barrier(2)
    slots = [None, None]
    results = {}

    def gather_for(r):
        def gather(rec):
            slots[r] = list(rec)
            barrier.wait()
            out = [list(slots[0]), list(slots[1])]
            barrier.wait()
            return out
        return gather

    def worker(r):
        results[r] = run_sharded(make_run(r), 4, gather_for(r), r)

    ts = [threading.Thread(target=worker, args=(r,)) for r in (0, 1)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert calls[0] == [4]
    assert calls[1] == [4, 14]                  # re-run from rank 0's lastIndex out
    assert results[1][0] == "out1@14" and results[1][1] == 34 and results[0][1] == 34


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, seed, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "oracle"), os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    import pyoracle
    from autoscaler_amd import shard
    from estgen import _encode_estimate, _estimate_inputs

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng, nodes, pods, templates, groups = _estimate_inputs(seed, n_groups=8, n_pods=60)
        table, node_recs, tm, off, pod_idx = _encode_estimate(nodes, pods, templates, groups)
        max_nodes = 0
        L0 = 3
        G = len(tm)
        a, b = rank * G // world, (rank + 1) * G // world
        off_blk = off[a:b + 1] - off[a]
        idx_blk = pod_idx[off[a]:off[b]]

        def run(lin):
            o = pyoracle.OracleState()
            if len(node_recs):
                o.add_nodes(node_recs)
            out = o.estimate(table, off_blk, idx_blk, tm[a:b], max_nodes, lin)
            # conservative: every block counts as lastIndex-sensitive with a success
            return out, out.last_index, 1, 1

        out, final_L, reruns = shard.run_sharded(run, L0, shard.torch_all_gather(dist, "cpu"), rank)
        # sequential reference over every group
        o = pyoracle.OracleState()
        if len(node_recs):
            o.add_nodes(node_recs)
        ref = o.estimate(table, off, pod_idx, tm, max_nodes, L0)
        ok = np.array_equal(out.results, ref.results[a:b])
        for g in range(a, b):
            n = int(ref.results[g]["n_scheduled"])
            s0, s1 = off[g] - off[a], off[g] - off[a] + n
            ok &= np.array_equal(out.sched_pod[s0:s1], ref.sched_pod[off[g]:off[g] + n])
            ok &= np.array_equal(out.sched_node[s0:s1], ref.sched_node[off[g]:off[g] + n])
        ok &= final_L == ref.last_index
        q.put((rank, bool(ok), reruns))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("seed", [0, 3, 7])
def test_sharded_estimate_gloo_world2(seed, oracle_lib):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, seed, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert all(ok for _, ok, _ in res), res


def _sweep_worker(rank, world, port, n_nodes, q):
    """FindNodesToRemove with the candidates in contiguous blocks (candidates
    shard like node groups, cluster.go:130-137), one per rank, the lastIndex chain fixed up
    by run_sharded; the CPU restatement runs each block (the protocol under test)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "oracle"), os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    import pyoracle
    from autoscaler_amd import shard
    from autoscaler_amd import workloads as W

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = W.c3(n_nodes=n_nodes)
        C = len(w.candidates)
        a, b = rank * C // world, (rank + 1) * C // world
        off = w.move_off[a:b + 1] - w.move_off[a]
        moves = w.move_pods[w.move_off[a]:w.move_off[b]]
        hints0 = np.full(len(w.table), -1, np.int32)
        o = pyoracle.OracleState()
        W.load_sweep(o, w)
        L0 = 11

        def run(lin):
            out = o.find_nodes_to_remove(w.candidates[a:b], w.dest_mask, w.cand_status[a:b], off, moves,
                                         hints0.copy(), lin)
            # a block whose scans all failed passes lastIndex through; count it sensitive
            # whenever it moved lastIndex (conservative: the protocol re-runs it)
            moved = int(out.last_index != lin)
            return out, out.last_index, 1, moved

        out, final_L, reruns = shard.run_sharded(run, L0, shard.torch_all_gather(dist, "cpu"), rank)
        ref = o.find_nodes_to_remove(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods,
                                     hints0.copy(), L0)
        ok = np.array_equal(out.results, ref.results[a:b])
        ok &= np.array_equal(out.dest, ref.dest[w.move_off[a]:w.move_off[b]])
        ok &= np.array_equal(out.hints[moves], ref.hints[moves])
        ok &= final_L == ref.last_index
        q.put((rank, bool(ok), reruns))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_nodes", [120, 400])
def test_sharded_sweep_gloo_world2(n_nodes, oracle_lib):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sweep_worker, args=(r, 2, port, n_nodes, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert all(ok for _, ok, _ in res), res
    assert res[1][2] >= 1                       # rank 1 re-ran from rank 0's lastIndex


def test_split_blocks_matches_library_rule():
    from autoscaler_amd.shard import split_blocks
    assert split_blocks([5, 5, 5, 5], 2) == [0, 2, 4]
    assert split_blocks([1, 1, 1], 5) == [0, 1, 2, 3, 3, 3]
    assert split_blocks([], 3) == [0, 0, 0, 0]
    b = split_blocks([30] * 100, 8)
    assert b[0] == 0 and b[-1] == 100 and len(b) == 9 and all(b[i] < b[i + 1] for i in range(8))


class _OracleBlockPlan:
    """A block's removal plan on the CPU restatement (test infrastructure): whole calls
    only (phased() False), as a plan with a prefix-protocol cut runs."""

    def __init__(self, o, w, a, b):
        self.o, self.w = o, w
        self.cand = w.candidates[a:b]
        self.status = w.cand_status[a:b]
        self.off = (w.move_off[a:b + 1] - w.move_off[a]).astype(np.int32)
        self.moves = w.move_pods[w.move_off[a]:w.move_off[b]]

    def sensitive_pods(self):
        return 0

    def phased(self):
        return False

    def run(self, lin, hints=None, want_dest=True):
        from autoscaler_amd import native
        ro = self.o.find_nodes_to_remove(self.cand, self.w.dest_mask, self.status, self.off, self.moves, hints.copy(),
                                         lin)
        hints[self.moves] = ro.hints[self.moves]
        return native.RemovalOutput(ro.results, ro.dest, hints, ro.last_index)


def _sweep_serial_worker(rank, world, port, n_nodes, q):
    """shard.sweep_sharded's whole-call path (blocks in order, one all-gather each) and its
    final exchange of results, destinations and hints, on the CPU restatement."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "oracle"), os.path.join(root, "tests")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    import pyoracle
    from autoscaler_amd import shard
    from autoscaler_amd import workloads as W

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w = W.c3(n_nodes=n_nodes)
        blocks = shard.split_blocks(np.diff(w.move_off), world)
        o = pyoracle.OracleState()
        W.load_sweep(o, w)
        plan = _OracleBlockPlan(o, w, blocks[rank], blocks[rank + 1])
        ex = shard.Exchange(shard.torch_gather_bytes(dist, "cpu"))
        sb, ph = shard.sweep_setup(plan, ex, rank, blocks[rank] == blocks[rank + 1])
        ok = True
        h_ref = np.full(len(w.table), -1, np.int32)
        hints = h_ref.copy()
        L = 11
        for loop in range(2):
            res, dest, final_L, st = shard.sweep_sharded(plan, L, hints, len(w.nodes), ex, rank, blocks, w.move_off,
                                                         w.move_pods, sb, ph)
            ref = o.find_nodes_to_remove(w.candidates, w.dest_mask, w.cand_status, w.move_off, w.move_pods, h_ref, L)
            ok &= np.array_equal(res, ref.results) and np.array_equal(dest, ref.dest)
            ok &= final_L == ref.last_index and np.array_equal(hints, ref.hints)
            ok &= st["serial_blocks"] == world
            h_ref, L = ref.hints.copy(), ref.last_index
        q.put((rank, bool(ok), 0))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_sweep_exchange_gloo(world, oracle_lib):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sweep_serial_worker, args=(r, world, port, 200, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res), res
