"""Per-kernel duration summary of a rocprofv3 --kernel-trace database
(python scripts/rocpd_stats.py <dir with *_results.db>)."""
import collections
import glob
import sqlite3
import sys

db = glob.glob(f"{sys.argv[1]}/*_results.db")[0]
c = sqlite3.connect(db)
t = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
kd = [x for x in t if x.startswith("rocpd_kernel_dispatch")][0]
ks = [x for x in t if x.startswith("rocpd_info_kernel_symbol")][0]
rows = c.execute(f"select s.display_name, d.end - d.start from {kd} d join {ks} s on d.kernel_id = s.id "
                 f"order by d.start").fetchall()
agg = collections.defaultdict(list)
for name, dur in rows:
    agg[name.split("(")[0]].append(dur / 1000)
print(f"{'kernel':44s} {'calls':>5s} {'mean_us':>9s} {'total_us':>9s}")
for name, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
    print(f"{name[:44]:44s} {len(v):5d} {sum(v) / len(v):9.1f} {sum(v):9.1f}")
