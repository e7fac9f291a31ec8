"""Recompute a bench line's roofline.frac from a rocprofv3 kernel_stats CSV (dev / evidence tool).
usage: python tools/frac_check.py <bench.json> <kernel_stats.csv> [<kernel_trace.csv> <warmup steps>]
The dominant kernel's rocprof name prefix is in roofline.kernel ("k_o2_j1=0 (k_o2<3, 3, 136, ...>)");
frac_rocprof = alg_flop_per_launch / AverageNs / peak.  Composite (staged) slots are skipped.
With the kernel trace of the same run: frac_rocprof_steady from the mean duration of the launches
after the warm-up steps (the stats' AverageNs includes the first launches, which run while the
GPU clocks ramp up -- 10-15 % slower -- and the bench line's mean is taken after its timed steps)."""
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
res = {"kernel": name, "calls": int(best["Calls"]), "avg_ms_rocprof": round(avg_ms, 4),
       "avg_ms_bench": r["avg_launch_ms"], "frac_bench": r["frac"],
       "frac_rocprof": round(frac, 5), "rel_diff": round(r["frac"] / frac - 1, 4)}
if len(sys.argv) > 4:
    skip = int(sys.argv[4]) * int(r.get("launches_per_step", 1))
    durs = [(int(t["End_Timestamp"]) - int(t["Start_Timestamp"])) / 1e6
            for t in csv.DictReader(open(sys.argv[3]))
            if re.sub(r"\(.*", "", t["Kernel_Name"]).replace("void ", "").replace("wstdev::", "")
            .startswith(name.rstrip(", "))][skip:]
    if durs:
        steady = sum(durs) / len(durs)
        fs = r["alg_flop_per_launch"] / (steady * 1e-3) / 1e12 / r["peak"]
        res.update({"steady_calls": len(durs), "avg_ms_rocprof_steady": round(steady, 4),
                    "frac_rocprof_steady": round(fs, 5), "rel_diff_steady": round(r["frac"] / fs - 1, 4)})
print(json.dumps(res))
