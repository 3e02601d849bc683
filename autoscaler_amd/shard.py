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
    """all_gather of a 4-int record over torch.distributed (RCCL or gloo)."""
    import torch

    def gather(rec):
        t = torch.tensor(rec, dtype=torch.int64, device=device)
        parts = [torch.empty_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(parts, t)
        return torch.stack(parts).cpu().tolist()
    return gather
