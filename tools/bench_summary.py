#!/usr/bin/env python3
"""Print the headline fields of a bench.py JSON line (used by the tools/gpu_r5*.sh scripts)."""
import json
import sys

d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("value %.4g  kernel %.2f us  frac %.3f  wall %.3f  cold %.3f" % (d["value"], r["kernel_ms_mean"] * 1e3, r["frac"],
                                                                    r["frac_wall"], r.get("frac_wall_cold", 0)))
for k in ("c3", "wide"):
    if k in d:
        print(k, {x: d[k][x] for x in ("ms_per_step", "frac_hbm") if x in d[k]})
if "rollout" in d:
    ro = d["rollout"]
    print("rollout %.2f us (random %.2f, planner shape %.2f)  likelihood %.3f ms  bounds %.3f ms" % (
        ro["ms_per_launch"] * 1e3, ro["random_order"]["ms_per_launch"] * 1e3,
        ro.get("planner_shape", {}).get("ms_per_launch", 0) * 1e3, ro["likelihood"]["ms_per_launch"],
        ro["subtask_bounds"]["ms_per_launch"]))
if "render" in d:
    print("render %.3f ms" % d["render"]["ms_per_launch"])
if d.get("cpu_baseline"):
    print("cpu_baseline %.3g (%d cores)" % (d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"]))
