"""One planner loop (canPersist=true) on C3 without a limit, for counter passes
(python scripts/planner_one.py [n_nodes]): scripts/planner_timing.run(n, 0, reps=1)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import planner_timing  # noqa: E402

planner_timing.run(int(sys.argv[1]) if len(sys.argv) > 1 else 5000, 0, reps=1)
