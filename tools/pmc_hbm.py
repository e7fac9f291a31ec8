"""HBM bytes per launch per kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE),
corrected as MI355X_MICROARCH.md prescribes (FETCH_SIZE x2 on gfx950; WRITE_SIZE as is; both in
KB units of 1024 B).  Also the ordered dispatch sequence [kernel, bytes] (the two passes run the
same launch sequence; paired by order), from which bench.py sums the kernels of a composite
timing slot (c5's HBM-staged levels).
usage: python tools/pmc_hbm.py <fetch_dir> <write_dir> <src_sha> <out.json>"""
import collections, csv, glob, json, os, re, sys


def dispatches(d, counter):
    """[(dispatch id, kernel, value)] in dispatch order (a counter's per-instance rows summed)."""
    acc = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            m = re.search(r"(k_[a-z0-9_]+<[^>]*>|k_big_[a-z]+)", r["Kernel_Name"])
            if m:
                key = int(r["Dispatch_Id"])
                name, v = acc.get(key, (m.group(1), 0.0))
                acc[key] = (name, v + float(r["Counter_Value"]))
    return [(k, n, v) for k, (n, v) in sorted(acc.items())]


def per_kernel(seq):
    vals = collections.defaultdict(list)
    for _, n, v in seq:
        vals[n].append(v)
    return vals


fseq = dispatches(sys.argv[1], "FETCH_SIZE")
wseq = dispatches(sys.argv[2], "WRITE_SIZE")
fetch = per_kernel(fseq)
write = per_kernel(wseq)
res = {"src_sha": sys.argv[3], "unit": "bytes per launch (mean over dispatches)",
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                 "FETCH_SIZE doubled (gfx950 half-count), KB = 1024 B",
       "hbm_bytes_per_launch": {}, "fetch_bytes_per_launch": {}, "write_bytes_per_launch": {},
       "dispatches": {}}
for k in sorted(set(fetch) | set(write)):
    f = 2 * 1024 * sum(fetch.get(k, [0])) / max(1, len(fetch.get(k, [])))
    w = 1024 * sum(write.get(k, [0])) / max(1, len(write.get(k, [])))
    res["fetch_bytes_per_launch"][k] = round(f)
    res["write_bytes_per_launch"][k] = round(w)
    res["hbm_bytes_per_launch"][k] = round(f + w)
    res["dispatches"][k] = len(fetch.get(k, []))
if [n for _, n, _ in fseq] == [n for _, n, _ in wseq]:
    res["dispatch_seq"] = [[n, round(2 * 1024 * f + 1024 * w)] for (_, n, f), (_, _, w) in zip(fseq, wseq)]
json.dump(res, open(sys.argv[4], "w"), indent=1)
print(json.dumps(res, indent=1))
