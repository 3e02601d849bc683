"""Chain phase per step from a rocprofv3 kernel trace (python scripts/rocprof_chain_span.py
<run_kernel_trace.csv>): the span from the first to the last end of each step's two
k_ffd_chain launches (heavy and light groups, overlapping) — what bench.py's
roofline.kernel_ms times with HIP events on the plan's stream."""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_ffd_chain" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
spans = [(max(d[i][1], d[i + 1][1]) - min(d[i][0], d[i + 1][0])) / 1e3 for i in range(0, len(d) - 1, 2)]
print(f"launches {len(d)}, steps {len(spans)}, chain span per step: mean {sum(spans) / len(spans):.1f} us, "
      f"min {min(spans):.1f}, max {max(spans):.1f}")
