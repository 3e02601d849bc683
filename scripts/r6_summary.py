"""One-screen summary of a bench.py JSON line (the legs' GPU / CPU-port times and ratios)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
x = d["extra"]
print(f"headline {d['ms_per_step']:.4f} ms  value {d['value']:.4g}  frac {d['roofline']['frac']:.4f}  "
      f"device_resident {x['device_resident']['ms_per_step']:.4f}  n_gpus {d['n_gpus']}")
if "sweep" in x:
    s = x["sweep"]
    print(f"sweep C3 fresh {s['fresh_ms']:.3f} ({s.get('fresh_speedup', 0):.1f}x) hinted {s['hinted_ms']:.3f} "
          f"({s.get('hinted_speedup', 0):.1f}x)")
if "c4" in x:
    print(f"c4 {x['c4']['estimate_ms']:.3f} ms ({x['c4'].get('speedup', 0):.0f}x)")
if "filter" in x:
    for k, v in x["filter"].items():
        if isinstance(v, dict) and "call_ms" in v:
            print(f"filter {k}: call {v['call_ms']:.2f} kernel {v['kernel_ms']:.2f} cpu {v.get('cpu_ms', 0):.2f} "
                  f"({v.get('speedup', 0):.2f}x) parity {v.get('parity')}")
if "utilization" in x:
    u = x["utilization"]
    print(f"util kernel {u['kernel_ms']:.4f} call {u['call_ms']:.4f} frac {u['roofline']['frac']:.3f}")
if "c5_runonce" in x:
    r = x["c5_runonce"]
    print("c5 gpu", {k: round(v, 3) for k, v in r["gpu_ms"].items()})
    print("c5 speedup", {k: round(v, 2) for k, v in r.get("speedup", {}).items()}, "parity", r.get("parity"))
if "planner" in x:
    for k, v in x["planner"]["runs"].items():
        print(f"planner limit {k}: gpu {v['gpu_ms']:.3f} cpu {v.get('cpu_ms', 0):.3f} ({v.get('speedup', 0):.2f}x) "
              f"parity {v.get('parity')}")
if "expansion" in x:
    e = x["expansion"]["groups"]
    print(f"expansion groups verdicts {e['verdicts_ms']:.4f} resident {e['resident_verdicts_ms']:.4f}")
for k in ("c3_multi", "c4_multi", "c5_runonce_multi"):
    if k in x:
        print(k, {a: b for a, b in x[k].items() if isinstance(b, (int, float, bool)) or a.startswith("results")})
