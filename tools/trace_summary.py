"""Per-kernel summary (name, calls, total / average microseconds as the database reports them) of a rocprofv3 kernel-trace database, the
framework's kernels only (names in namespace fa::).  Usage: python tools/trace_summary.py RUN_DIR [OUT_CSV]"""
import csv
import glob
import sqlite3
import sys


def main():
    db = glob.glob(f"{sys.argv[1]}/**/*.db", recursive=True)[0]
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("pragma table_info(top_kernels)")]
    rows = [dict(zip(cols, r)) for r in con.execute("select * from top_kernels")]
    rows = [r for r in rows if "fa::" in r["name"]]
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["name", "calls", "total_us", "average_us"])
    for r in rows:
        w.writerow([r["name"], r["total_calls"], round(r["total_duration"], 1), round(r["average"], 1)])


if __name__ == "__main__":
    main()
