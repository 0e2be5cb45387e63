#!/usr/bin/env python3
"""Per-kernel PMC summary of the scripts/pmc.sh passes (rocprofv3 --pmc, CSV output).

Averages every counter per dispatch of each kernel and derives HBM traffic the way
MI355X_MICROARCH.md prescribes for gfx950: FETCH_SIZE (KiB) is under-reported by 2x, so
bytes read = 2 * FETCH_SIZE * 1024; bytes written = WRITE_SIZE * 1024.

Usage: pmc_summary.py <pmc dir (gpurun_out/pmc_<tag>)> <out.csv>
"""
import collections
import csv
import glob
import os
import sys


def load(pattern):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(pattern):
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r["Kernel_Name"].split("(")[0]
                if "rocprim" in name:
                    name = "rocprim::" + ("scan" if "scan" in name else "sort" if "sort" in name else "prim")
                acc[name][(r["Counter_Name"], r["Dispatch_Id"])].append(float(r["Counter_Value"]))
    out = {}
    for name, d in acc.items():
        per = collections.defaultdict(list)
        for (cn, _), vals in d.items():
            per[cn].append(sum(vals))  # one value per dispatch (summed over dimensions)
        out[name] = {cn: sum(v) / len(v) for cn, v in per.items()}
        out[name]["DISPATCHES"] = max(len(v) for v in per.values())
    return out


def main():
    base, dst = sys.argv[1], sys.argv[2]
    data = collections.defaultdict(dict)
    for sub in ("sq", "fetch", "write"):
        for k, v in load(os.path.join(base, sub, "*counter_collection.csv")).items():
            data[k].update(v)
    cols = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAIT_INST_LDS",
            "SQ_LDS_BANK_CONFLICT", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "FETCH_SIZE", "WRITE_SIZE"]
    rows = []
    for k, v in data.items():
        rd = 2 * v.get("FETCH_SIZE", 0.0) * 1024
        wr = v.get("WRITE_SIZE", 0.0) * 1024
        rows.append([k] + [round(v.get(c, 0.0), 1) for c in cols] + [round(rd), round(wr), round(rd + wr), int(v.get("DISPATCHES", 1))])
    rows.sort(key=lambda r: -r[-2])
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel"] + [c.lower() for c in cols] + ["hbm_read_bytes", "hbm_write_bytes", "hbm_bytes", "dispatches"])
        w.writerows(rows)
    for r in rows[:25]:
        print(r[0][:28].ljust(28), " ".join(str(x) for x in r[1:]))


if __name__ == "__main__":
    main()
