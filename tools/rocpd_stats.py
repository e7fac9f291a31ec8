"""Per-kernel duration summary (rocprofv3 --stats layout) from a rocprofv3 rocpd SQLite database,
for runs made without --output-format csv.  usage: python tools/rocpd_stats.py <dir_or_db> <out.csv>"""
import csv, glob, os, sqlite3, sys

src = sys.argv[1]
db = src if src.endswith(".db") else glob.glob(os.path.join(src, "**", "*.db"), recursive=True)[0]
con = sqlite3.connect(db)
rows = con.execute(
    "select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
# rocpd's top_kernels reports microseconds; the csv --stats layout is nanoseconds
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
    for name, calls, tot, avg, pct in rows:
        w.writerow([name, calls, round(tot * 1e3), round(avg * 1e3, 3), round(pct, 4)])
print(open(sys.argv[2]).read())
