#!/usr/bin/env python3
"""Top kernels of a rocprofv3 --stats kernel_stats.csv: prof_top.py <csv> [n]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
for r in rows[:n]:
    print("%-55s %5s %10.1f us" % (r["Name"][:55], r["Calls"], float(r["AverageNs"]) / 1e3))
