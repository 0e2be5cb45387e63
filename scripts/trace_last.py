"""The kernels of the last merge in a rocprofv3 kernel trace (from the last k_spec / k_direct /
k_wlen launch on), with their start offsets and durations in us; `min_us` filters short ones."""
import csv
import glob
import sys

d, min_us = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
if f:
    r = list(csv.DictReader(open(f[0])))
else:  # rocprofv3's default rocpd database
    import sqlite3
    db = sqlite3.connect(glob.glob(f"{d}/**/*.db", recursive=True)[0])
    r = [{"Kernel_Name": n, "Start_Timestamp": a, "End_Timestamp": b, "Stream": st}
         for n, a, b, st in db.execute("select name, start, end, stream from kernels")]
r = sorted(r, key=lambda x: int(x["Start_Timestamp"]))
starts = [i for i, x in enumerate(r) if "k_fill_multi" in x["Kernel_Name"]]
a = starts[-1] if starts else 0
# the last merge starts at the fill of its decode counters: find the fill before the last k_spec / k_direct
first = [i for i, x in enumerate(r) if any(k in x["Kernel_Name"] for k in ("k_spec", "k_direct(", "k_wlen"))]
if first:
    b = first[-1]
    a = max([i for i in starts if i <= b] or [b])
t0 = int(r[a]["Start_Timestamp"])
tot = {}
for x in r[a:]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    name = x["Kernel_Name"].split("(")[0][:60]
    tot[name] = tot.get(name, 0.0) + (e - s) / 1e3
    if (e - s) / 1e3 >= min_us:
        print("%10.1f %9.1f %s %s" % ((s - t0) / 1e3, (e - s) / 1e3, name, x.get("Stream", "")))
print("last merge: %.1f us from first to last kernel end; %d dispatches" % ((int(r[-1]["End_Timestamp"]) - t0) / 1e3, len(r) - a))
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:12]:
    print("  %9.1f us  %s" % (v, k))
