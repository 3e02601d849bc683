"""One-screen summary of a bench.py JSON line (python scripts/bench_summary.py FILE)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d["extra"]
print("headline ms", round(d["ms_per_step"], 4), "value", f"{d['value']:.3e}", "frac", round(d["roofline"]["frac"], 4))
print("device", round(e["device_resident"]["ms_per_step"], 4), "i32", (e.get("host_int32_ids") or {}).get("ms_per_step"))
if e.get("cold"):
    print("cold", {k: round(v, 3) for k, v in e["cold"].items() if isinstance(v, float)})
if "sweep" in e:
    print("sweep", {k: round(e["sweep"][k], 3) for k in ("fresh_ms", "hinted_ms", "fresh_speedup", "hinted_speedup")})
if "c5_runonce" in e:
    r = e["c5_runonce"]
    print("runonce gpu", {k: round(v, 3) for k, v in r["gpu_ms"].items()})
    print("runonce cpu", {k: round(v, 3) for k, v in r["cpu_ms"].items()}, "parity", all(r["parity"].values()))
if "planner" in e:
    print("planner", {k: (round(v["gpu_ms"], 3), round(v.get("cpu_ms", 0), 3), v.get("parity")) for k, v in e["planner"]["runs"].items()})
    for k, v in e["planner"]["runs"].items():
        if "split_ms" in v:
            print("  planner", k, {x: round(y, 3) for x, y in v["split_ms"].items()})
if "filter" in e:
    print("filter", {k: (round(e["filter"][k]["call_ms"], 2), round(e["filter"][k]["cpu_ms"], 2)) for k in ("c5", "c5-c4")})
for k in ("c4", "c2_unlimited", "utilization"):
    if k in e:
        v = e[k]
        print(k, {x: v[x] for x in ("estimate_ms", "ms_per_step", "kernel_ms", "call_ms", "cpu_ms", "speedup", "parity", "parity_vs_golden") if x in v})
