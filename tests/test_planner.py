"""Planner.categorizeNodes with canPersist=true on the CPU: the oracle's
loop (or_plan_removals) against the step-by-step restatement of tests/plangen.py, and
the reference's planner_test.go known answers through the Python Planner."""
from __future__ import annotations

import numpy as np
import pytest

from plangen import node_states, plan_by_steps, rand_plan_case


def _same(a, b, what):
    assert np.array_equal(a, b), (what, a, b)


@pytest.mark.parametrize("seed", range(40))
def test_oracle_plan_matches_steps(seed, oracle_lib):
    oracle = oracle_lib
    case = rand_plan_case(seed, n_nodes=10 + seed % 7, pods_per_node=3 + seed % 3, n_pdbs=(seed % 3) * 2)
    a = oracle.OracleState()
    case.load(a)
    got = case.plan(a)
    b = oracle.OracleState()
    case.load(b)
    want = plan_by_steps(b, case)
    _same(got.results, want["results"], "results")
    _same(got.moves, want["moves"], "moves")
    _same(got.hints, want["hints"], "hints")
    assert got.last_index == want["last_index"]
    _same(got.allowed, want["allowed"], "pdb budgets")
    assert node_states(a, len(case.node_recs)) == node_states(b, len(case.node_recs))


def test_oracle_plan_commits_feed_later_candidates(oracle_lib):
    oracle = oracle_lib
    """A removable candidate's copies land on a later candidate, which must then move them
    too (its pods to move grow), and a removed node is no destination for later ones."""
    hits = 0
    for seed in range(60):
        case = rand_plan_case(seed, n_nodes=8, pods_per_node=4, limit=0)
        a = oracle.OracleState()
        case.load(a)
        out = case.plan(a)
        cand_pos = {int(c): k for k, c in enumerate(case.cands)}
        for mv in out.moves:
            k = cand_pos.get(int(mv["node"]))
            if k is not None and k > mv["candidate"] and out.results[k]["reason"] in (0, 12):
                hits += 1
                r = out.results[k]
                own = case.off[k + 1] - case.off[k]
                assert r["removable"] == 0 or r["n_moves"] > own
        for mv in out.moves:                       # planner.go:280: removed nodes are no destination
            assert int(mv["node"]) not in {int(case.cands[k]) for k in range(mv["candidate"] + 1)
                                           if out.results[k]["removable"]}
    assert hits > 0
