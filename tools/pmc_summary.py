"""Aggregate rocprofv3 --pmc CSVs per kernel instantiation (dev tool)."""
import collections, csv, glob, os, sys
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if "rocclr" in name:
            continue
        short = name.replace("void (anonymous namespace)::", "").split("(")[0]
        # counters that appear in several passes (SQ_WAVES, SQ_BUSY_CYCLES) are kept per pass file
        # and averaged below, not summed over the passes
        agg[short][(r["Counter_Name"], f)] += float(r["Counter_Value"])
        disp[short].add(r["Dispatch_Id"])
for k in agg:
    per = collections.defaultdict(list)
    for (n, f), v in agg[k].items():
        per[n].append(v)
    agg[k] = {n: sum(v) / len(v) for n, v in per.items()}
for k in sorted(agg):
    c = agg[k]
    w = c.get("SQ_WAVES", 0) or 1
    print(f"== {k}  dispatches/pass~{len(disp[k])//3 or len(disp[k])}")
    for n in sorted(c):
        print(f"   {n:28s} {c[n]:.4e}   per-wave {c[n]/w:.1f}")
    if "SQ_INSTS_VALU" in c:
        v = c["SQ_INSTS_VALU"]
        print(f"   VALU mix: int32 {c.get('SQ_INSTS_VALU_INT32',0)/v:.2%} fma {c.get('SQ_INSTS_VALU_FMA_F32',0)/v:.2%} "
              f"add {c.get('SQ_INSTS_VALU_ADD_F32',0)/v:.2%} mul {c.get('SQ_INSTS_VALU_MUL_F32',0)/v:.2%}")
    if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
        print(f"   LDS conflict cycles / LDS active: {c['SQ_LDS_BANK_CONFLICT']/c['SQ_LDS_IDX_ACTIVE']:.2%}")
    if c.get("SQ_WAVE_CYCLES"):
        wc = c["SQ_WAVE_CYCLES"]
        print("   share of wave cycles: " + " ".join(
            f"{n[3:].lower()} {c[n] / wc:.2%}" for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS",
                                                       "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU") if n in c))
