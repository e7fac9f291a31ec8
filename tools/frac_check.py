"""Recompute a bench line's roofline.frac from a rocprofv3 kernel_stats CSV (dev / evidence tool).
usage: python tools/frac_check.py <bench.json> <kernel_stats.csv>
The dominant kernel's rocprof name prefix is in roofline.kernel ("k_o2_j1=0 (k_o2<3, 3, 136, ...>)");
frac_rocprof = alg_flop_per_launch / AverageNs / peak.  Composite (staged) slots are skipped."""
import csv
import json
import re
import sys

line = json.load(open(sys.argv[1]))
r = line["roofline"]
m = re.search(r"\((k_\w+<[^.]*?)(?:, \.\.\.>|\.\.\.>|>)\)", r["kernel"])
name = m.group(1) if m else None
if not name or "+" in r["kernel"]:
    print(json.dumps({"kernel": r["kernel"], "frac_bench": r["frac"], "frac_rocprof": None,
                      "note": "composite slot: no single kernel"}))
    sys.exit(0)
best = None
for row in csv.DictReader(open(sys.argv[2])):
    short = re.sub(r"\(.*", "", row["Name"]).replace("void ", "").replace("wstdev::", "")
    if short.startswith(name.rstrip(", ")) and (best is None or int(row["Calls"]) > int(best["Calls"])):
        best = row
if best is None:
    print(json.dumps({"kernel": name, "frac_bench": r["frac"], "frac_rocprof": None, "note": "not in CSV"}))
    sys.exit(1)
avg_ms = float(best["AverageNs"]) / 1e6
ach = r["alg_flop_per_launch"] / (avg_ms * 1e-3) / 1e12
frac = ach / r["peak"]
print(json.dumps({"kernel": name, "calls": int(best["Calls"]), "avg_ms_rocprof": round(avg_ms, 4),
                  "avg_ms_bench": r["avg_launch_ms"], "frac_bench": r["frac"],
                  "frac_rocprof": round(frac, 5), "rel_diff": round(r["frac"] / frac - 1, 4)}))
