"""Print average kernel durations from rocprofv3 kernel_stats CSVs (dev tool).
usage: python tools/kstats.py <regex> <dir-or-csv> ..."""
import csv, glob, os, re, sys
rx = re.compile(sys.argv[1])
for d in sys.argv[2:]:
    f = d if d.endswith('.csv') else (glob.glob(os.path.join(d, '**', '*kernel_stats.csv'), recursive=True) or [''])[0]
    if not f:
        print(f"{d}: no stats"); continue
    rows = list(csv.DictReader(open(f)))
    out = []
    for r in rows:
        if rx.search(r['Name']):
            name = re.sub(r'\(.*', '', r['Name']).replace('void wstdev::', '')
            out.append("%8.1fus %s" % (float(r['AverageNs']) / 1e3, name))
    print("%-28s: %s" % (os.path.basename(d.rstrip('/')), " | ".join(out)))
