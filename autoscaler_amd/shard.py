"""Node-group sharding across ranks (one process per GPU) with the lastIndex chain.

SURVEY.md §8e: node groups are split into contiguous blocks, one per rank, and the
blocks are coupled only through the checker's lastIndex
(CA/simulator/predicatechecker/schedulerbased.go:43,131).  Each rank runs its block
from the caller's lastIndex; one all_gather of a 4-int record per rank
(lastIndex in, lastIndex out, lastIndex-sensitive, had a FitsAnyNode success) lets every
rank walk the chain in rank order.  The first rank whose block is lastIndex-sensitive
and was run from a wrong input re-runs from the exact value; repeat until the walk
accepts every block (at most `world` rounds; on C2 none, since a block's first success
happens with one new node).  No other data crosses ranks.
"""
from __future__ import annotations

from typing import Callable, Tuple


def walk(records, L0: int) -> Tuple[int, int]:
    """Walk per-rank records (lin, lout, sensitive, had_success) in rank order from L0.
    Returns (first rank to re-run or -1, exact lastIndex before it / after all)."""
    cur = L0
    for r, (l_in, l_out, sens, succ) in enumerate(records):
        if l_in != cur and sens:
            return r, cur
        cur = l_out if succ else cur
    return -1, cur


def run_sharded(run: Callable[[int], Tuple[object, int, int, int]], L0: int, all_gather: Callable[[list], list],
                rank: int) -> Tuple[object, int, int]:
    """Run this rank's block and fix up the lastIndex chain.

    run(lin) -> (output, lout, sensitive, had_success) for this rank's block.
    all_gather(rec) -> list of every rank's 4-int record, in rank order.
    Returns (output, final lastIndex after the last rank, number of re-runs here)."""
    lin = L0
    out, lout, sens, succ = run(lin)
    reruns = 0
    while True:
        recs = all_gather([lin, lout, sens, succ])
        bad, cur = walk(recs, L0)
        if bad < 0:
            return out, cur, reruns
        if bad == rank:
            lin = cur
            out, lout, sens, succ = run(lin)
            reruns += 1


def torch_all_gather(dist, device) -> Callable[[list], list]:
    """all_gather of a 4-int record over torch.distributed (RCCL or gloo).  The tensors are
    allocated once (a step of the C2 headline is ~0.5 ms: per-call allocations and the
    list form's stack cost a noticeable share of it); one H2D copy in, one D2H copy out."""
    import torch
    world = dist.get_world_size()
    src = torch.zeros(4, dtype=torch.int64, device=device)
    parts = [torch.zeros(4, dtype=torch.int64, device=device) for _ in range(world)]
    flat = torch.zeros(4 * world, dtype=torch.int64, device=device)
    into = str(device) != "cpu" and hasattr(dist, "all_gather_into_tensor")

    def gather(rec):
        src.copy_(torch.tensor(rec, dtype=torch.int64))
        if into:
            dist.all_gather_into_tensor(flat, src)
            v = flat.cpu().tolist()
        else:
            dist.all_gather(parts, src)
            v = [x for p in parts for x in p.tolist()]
        return [v[4 * r:4 * r + 4] for r in range(world)]
    return gather


# ---- blocks, byte all-gathers, and the chained batches of one process per GPU -------------

def split_blocks(weights, world: int) -> list:
    """Contiguous blocks of units [0, n), one per rank, balanced by weight (each weight at
    least 1): the split multi.hip's split_blocks makes, so the one-process-per-GPU form and
    the library's multi-device form run the same blocks.  Returns world + 1 bounds (trailing
    empty blocks when there are fewer units than ranks)."""
    import numpy as np
    w = np.maximum(np.asarray(weights, dtype=np.int64), 1)
    n = len(w)
    b = [0]
    if n > 0:
        D = max(1, min(world, n))
        tot, acc = int(w.sum()), 0
        for i in range(n):
            acc += int(w[i])
            k = len(b)
            if k < D and i + 1 < n and n - (i + 1) >= D - k and acc * D >= tot * k:
                b.append(i + 1)
    b.append(n)
    while len(b) < world + 1:
        b.append(n)
    return b


def torch_gather_bytes(dist, device) -> Callable:
    """all_gather of an equal-sized numpy array per rank (any dtype, moved as bytes) over
    torch.distributed (RCCL over xGMI, or gloo): returns every rank's array, in rank order."""
    import numpy as np
    import torch

    def gather(arr):
        a = np.ascontiguousarray(arr)
        t = torch.from_numpy(a.reshape(-1).view(np.uint8).copy()).to(device)
        parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, t)
        return [p.cpu().numpy().view(a.dtype).reshape(a.shape) for p in parts]
    return gather


class Exchange:
    """The collectives of one batch, counted: every rank's record in rank order
    (``gather``), and the bytes this rank contributed (``bytes``, ``calls``)."""

    def __init__(self, gather_bytes: Callable):
        self._g = gather_bytes
        self.bytes = 0
        self.calls = 0

    def gather(self, arr):
        import numpy as np
        a = np.ascontiguousarray(arr)
        self.bytes += a.nbytes
        self.calls += 1
        return self._g(a)


def _padded(arr, n: int, fill=0):
    import numpy as np
    out = np.full(n, fill, dtype=arr.dtype) if arr.dtype.fields is None else np.zeros(n, arr.dtype)
    out[: len(arr)] = arr
    return out


def chain_sharded(run: Callable, L0: int, all_gather: Callable, rank: int):
    """run_sharded, also returning the exact input lastIndex of this rank's block and the
    one its accepted run started from.  Returns (output, exact input, input used, final
    lastIndex, re-runs here)."""
    lin = L0
    out, lout, sens, succ = run(lin)
    reruns = 0
    while True:
        recs = all_gather([lin, lout, sens, succ])
        bad, cur = walk(recs, L0)
        if bad < 0:
            exact = L0
            for l_in, l_out, _s, sc in recs[:rank]:
                exact = l_out if sc else exact
            return out, exact, lin, cur, reruns
        if bad == rank:
            lin = cur
            out, lout, sens, succ = run(lin)
            reruns += 1


def estimate_sharded(plan, max_nodes: int, L0: int, ex: Exchange, rank: int, blocks, group_off,
                     assemble: bool = True):
    """Estimate over node groups in contiguous blocks, one per rank (the
    reference calls Estimate group after group with one checker, orchestrator.go:139-178):
    this rank's `plan` (native.EstimatePlan over groups [blocks[rank], blocks[rank+1]))
    runs from L0; the 4-int chain records are all-gathered (a lastIndex-sensitive block run
    from a wrong input runs again from the exact one); a block that ran from a wrong input
    without depending on it has its lastIndex fields re-based (ca_estimate_plan_rebase).
    With `assemble`, two more all-gathers bring every rank the whole batch's per-group
    records and scheduled pods.  Returns (results, sched_pod, final lastIndex,
    re-runs here) — the whole batch's with `assemble`, else this block's."""
    import numpy as np
    from . import abi
    g0, g1 = blocks[rank], blocks[rank + 1]

    def run(lin):
        if g1 == g0:
            return None, lin, 0, 0
        out = plan.run(max_nodes, lin, want_nodes=False, copy=True)
        sens, succ = plan.chain_info()
        return out, out.last_index, sens, succ

    def gather4(rec):
        return [[int(v) for v in r] for r in ex.gather(np.array(rec, np.int64))]

    out, exact, used, final_L, reruns = chain_sharded(run, L0, gather4, rank)
    res = out.results if out is not None else np.zeros(0, abi.ESTIMATE_RESULT_DTYPE)
    sched = out.sched_pod if out is not None else np.zeros(0, np.int32)
    if out is not None and used != exact:
        res = res.copy()
        plan.rebase(res, exact)
    if not assemble:
        return res, sched, final_L, reruns
    R = len(blocks) - 1
    G = len(group_off) - 1
    nmax = max(1, max(int(group_off[blocks[r + 1]] - group_off[blocks[r]]) for r in range(R)))
    gmax = max(1, max(blocks[r + 1] - blocks[r] for r in range(R)))
    recs_all = ex.gather(_padded(res, gmax))
    sched_all = ex.gather(_padded(np.ascontiguousarray(sched, np.int32), nmax, -1))
    full_res = np.zeros(G, abi.ESTIMATE_RESULT_DTYPE)
    full_sched = np.full(int(group_off[-1]), -1, np.int32)
    for r in range(R):
        a, b = blocks[r], blocks[r + 1]
        full_res[a:b] = recs_all[r][: b - a]
        ia, ib = int(group_off[a]), int(group_off[b])
        full_sched[ia:ib] = sched_all[r][: ib - ia]
    return full_res, full_sched, final_L, reruns


def sweep_sharded(plan, L0: int, hints, n_nodes: int, ex: Exchange, rank: int, blocks, move_off, move_pods,
                  sens_before: int, phased: bool, assemble: bool = True):
    """FindNodesToRemove over candidates in contiguous blocks, one per rank (SURVEY §8e;
    cluster.go:130-137 walks the candidates in order with one checker), in the three
    phases of casim.h "one process per GPU": PROBE, all-gather of the 560-B records, MAP,
    all-gather, ca_sweep_compose (every rank composes the same chain), RESOLVE from the
    block's exact input.  Blocks the maps do not reach (or every block when some plan has a
    prefix-protocol cut: `phased` False on any rank) run whole calls in order, each from
    its predecessor's output (one all-gather per block).  `plan`: native.RemovalPlan over
    this rank's candidates; `hints`: this rank's per-pod hint array (caller-held, int32),
    updated for every block's pods by the final exchange; `sens_before`: the pods to move
    of the earlier blocks' lastIndex-sensitive candidates (ca_removal_plan_sensitive_pods,
    gathered once per plan set: ``sweep_setup``).

    Returns (results, dest, final lastIndex, stats) — with `assemble` the whole call's
    results and destinations (one more all-gather, which also carries the hints of every
    block's pods), else this block's."""
    import numpy as np
    from . import abi, native
    R = len(blocks) - 1
    c0, c1 = blocks[rank], blocks[rank + 1]
    empty = c1 == c0
    stats = {"reached": R, "serial_blocks": 0}
    rec = np.zeros(1, abi.SWEEP_PHASE_DTYPE)
    out = None
    lin_c = np.full(R, abi.CA_SWEEP_NOT_REACHED, np.int32)
    all_phased = bool(np.all([int(v[0]) for v in ex.gather(np.array([1 if (phased or empty) else 0], np.int32))]))
    if all_phased and n_nodes > 0 and R > 1:
        rec["kind"] = abi.CA_SWEEP_PHASE_PROBE
        rec["guess_base"] = int(L0) + int(sens_before)
        if not empty:
            plan.run_phase(rec, hints, L0, want_dest=False)
        probes = np.concatenate(ex.gather(rec))
        est = int(L0) + int(probes["adv"][:rank].sum())
        rec["kind"] = abi.CA_SWEEP_PHASE_MAP
        rec["est_base"] = est % n_nodes
        if not empty and int(rec["n_sensitive"][0]) > 0:
            plan.run_phase(rec, hints, L0, want_dest=False)
        maps = np.concatenate(ex.gather(rec))
        lin_c = native.sweep_compose(maps, n_nodes, L0)
        if lin_c[rank] != abi.CA_SWEEP_NOT_REACHED and not empty:
            rec["kind"] = abi.CA_SWEEP_PHASE_RESOLVE
            out = plan.run_phase(rec, hints, int(lin_c[rank]), want_dest=True)
        stats["reached"] = int((lin_c != abi.CA_SWEEP_NOT_REACHED).sum())
    # the chain through the composed blocks, then whole calls in order for the rest
    r0 = int(np.argmax(lin_c == abi.CA_SWEEP_NOT_REACHED)) if (lin_c == abi.CA_SWEEP_NOT_REACHED).any() else R
    cur = int(L0)
    if r0 > 0:                             # the exact output of the last reached block
        louts = ex.gather(np.array([out.last_index if out is not None else int(lin_c[rank])], np.int64))
        cur = int(louts[r0 - 1][0])
    cut = False
    for r in range(r0, R):
        if r == rank and not empty:
            if cut:
                res = np.zeros(c1 - c0, abi.REMOVAL_RESULT_DTYPE)
                res["reason"] = abi.CA_UNREMOVABLE_NOT_RUN
                res["last_index_in"] = cur
                out = native.RemovalOutput(res, np.full(int(move_off[c1] - move_off[c0]), -1, np.int32), hints, cur)
            else:
                out = plan.run(cur, hints=hints, want_dest=True)
        stats["serial_blocks"] += 1
        msg = ex.gather(np.array([out.last_index if (r == rank and out is not None) else 0,
                                  int(r == rank and out is not None and not cut and
                                      bool((out.results["reason"] == abi.CA_UNREMOVABLE_OUT_OF_SCOPE).any()))],
                                 np.int64))
        if blocks[r + 1] > blocks[r]:
            cur = int(msg[r][0])
            cut = cut or bool(msg[r][1])
    if not assemble:
        return (out.results if out is not None else np.zeros(0, abi.REMOVAL_RESULT_DTYPE),
                out.dest if out is not None else np.zeros(0, np.int32), cur, stats)
    # one all-gather: every block's results, destinations and its pods' hints
    C = len(move_off) - 1
    cmax = max(1, max(blocks[r + 1] - blocks[r] for r in range(R)))
    mmax = max(1, max(int(move_off[blocks[r + 1]] - move_off[blocks[r]]) for r in range(R)))
    res = out.results if out is not None else np.zeros(0, abi.REMOVAL_RESULT_DTYPE)
    dest = out.dest if out is not None else np.zeros(0, np.int32)
    mine = np.asarray(move_pods[int(move_off[c0]):int(move_off[c1])], np.int64)
    rec_b = np.zeros(1, np.dtype([("res", abi.REMOVAL_RESULT_DTYPE, (cmax,)), ("dest", np.int32, (mmax,)),
                                  ("hint", np.int32, (mmax,))]))
    rec_b["res"][0][: len(res)] = res
    rec_b["dest"][0][:] = -1
    rec_b["dest"][0][: len(dest)] = dest
    rec_b["hint"][0][: len(mine)] = hints[mine]
    parts = ex.gather(rec_b)
    full_res = np.zeros(C, abi.REMOVAL_RESULT_DTYPE)
    full_dest = np.full(int(move_off[-1]), -1, np.int32)
    for r in range(R):
        a, b = blocks[r], blocks[r + 1]
        ma, mb = int(move_off[a]), int(move_off[b])
        full_res[a:b] = parts[r]["res"][0][: b - a]
        full_dest[ma:mb] = parts[r]["dest"][0][: mb - ma]
        if r != rank:
            hints[np.asarray(move_pods[ma:mb], np.int64)] = parts[r]["hint"][0][: mb - ma]
    stats["collective_bytes"] = ex.bytes
    stats["collectives"] = ex.calls
    return full_res, full_dest, cur, stats


def sweep_setup(plan, ex: Exchange, rank: int, empty: bool):
    """Once per set of block plans: (sens_before, phased) for sweep_sharded — the pods to
    move of the earlier blocks' sensitive candidates (the probe's guess step) and whether
    this block's plan can run the phases (no prefix-protocol cut)."""
    import numpy as np
    mine = 0 if empty else plan.sensitive_pods()
    allv = ex.gather(np.array([mine], np.int64))
    return int(sum(int(v[0]) for v in allv[:rank])), (True if empty else plan.phased())
