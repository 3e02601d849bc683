"""Print a rocprofv3 kernel_trace.csv as a timeline (sorted by start), with gaps between
dispatches: python scripts/trace_timeline.py <run_kernel_trace.csv> [first] [count]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
count = int(sys.argv[3]) if len(sys.argv) > 3 else len(rows)
prev_end = None
t0 = int(rows[first]["Start_Timestamp"]) if rows else 0
for i, r in enumerate(rows[first:first + count], first):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = "" if prev_end is None else f"gap {(s - prev_end) / 1e3:8.2f}"
    print(f"{i:5d} t={(s - t0) / 1e3:10.2f}us dur {(e - s) / 1e3:8.2f}us {gap}  "
          f"{r['Kernel_Name'].split('(')[0][:34]:34s} grid {r['Grid_Size_X']}x{r['Grid_Size_Y']} wg {r['Workgroup_Size_X']}")
    prev_end = e
