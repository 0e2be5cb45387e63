#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (results.db or kernel_stats.csv) into a CSV
under profiles/: kernel, calls, total_us, avg_us, pct. Usage: prof_summary.py <db|csv> <out.csv>"""
import csv
import sqlite3
import sys


def rows_from_db(path):
    c = sqlite3.connect(path)
    for name, calls, total, avg, pct in c.execute(
            "select name,total_calls,total_duration,average,percentage from top_kernels"):
        yield name, calls, total, avg, pct  # the rocpd top_kernels view is already in us


def rows_from_csv(path):
    with open(path) as f:
        for r in csv.DictReader(f):
            yield (r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                   float(r["AverageNs"]) / 1e3, float(r["Percentage"]))


def short(name):
    if "rocprim" in name:
        kind = "scan" if "scan" in name else "sort" if "sort" in name else "prim"
        return f"rocprim::{kind}::" + ("init_lookback" if "init_lookback" in name else "kernel")
    return name.split("(")[0]


def main():
    src, dst = sys.argv[1], sys.argv[2]
    rows = list(rows_from_db(src) if src.endswith(".db") else rows_from_csv(src))
    agg = {}
    for n, calls, tot, avg, pct in rows:
        k = short(n)
        a = agg.setdefault(k, [0, 0.0, 0.0])
        a[0] += calls
        a[1] += tot
        a[2] += pct
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "pct"])
        for k, (calls, tot, pct) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            w.writerow([k, calls, round(tot, 3), round(tot / calls, 3), round(pct, 2)])
    print(open(dst).read()[:2000])


if __name__ == "__main__":
    main()
