#!/usr/bin/env python3
"""Per-kernel read-request sizes from a rocprofv3 --pmc pass over TCC_EA0_RDREQ{,_32B,_64B,_128B}
(scripts/gpu_rdreq.sh): averages per dispatch and the fetched bytes they imply,
32 * n32 + 64 * n64 + 128 * n128 (requests of other sizes counted at 64 B).
Usage: rdreq_summary.py <pmc dir> <out.csv>"""
import collections
import csv
import glob
import os
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for path in glob.glob(os.path.join(sys.argv[1], "*counter_collection.csv")):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0]
        if "rocprim" in name:
            name = "rocprim::" + ("scan" if "scan" in name else "sort" if "sort" in name else "prim")
        acc[name][r["Counter_Name"].replace("_sum", "")] += float(r["Counter_Value"])
        disp[name].add(r["Dispatch_Id"])
rows = []
for k, d in acc.items():
    n = len(disp[k])
    tot, n32, n64, n128 = (d.get("TCC_EA0_RDREQ" + s, 0.0) / n for s in ("", "_32B", "_64B", "_128B"))
    other = max(0.0, tot - n32 - n64 - n128)
    rows.append([k, round(tot), round(n32), round(n64), round(n128), round(32 * n32 + 64 * n64 + 128 * n128 + 64 * other)])
rows.sort(key=lambda r: -r[-1])
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["kernel", "rdreq", "rdreq_32b", "rdreq_64b", "rdreq_128b", "read_bytes"])
    w.writerows(rows)
for r in rows:
    print(r[0][:32].ljust(32), *r[1:])
print("total read bytes per dispatch-set:", sum(r[-1] for r in rows))
