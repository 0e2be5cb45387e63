set -u
mkdir -p gpurun_out/sl
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sl -o sl -- python3 scripts/probe_small_large2.py 1 > gpurun_out/sl/probe.log 2>&1 || { tail -20 gpurun_out/sl/probe.log; exit 1; }
grep "PREDECODE" gpurun_out/sl/probe.log
f=$(find gpurun_out/sl -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
pre = [i for i, r in enumerate(rows) if "k_predecoded" in r["Kernel_Name"]]
a, z = pre[-2], pre[-1]
agg = collections.OrderedDict()
for r in rows[a - 5:z - 5]:
    n = r["Kernel_Name"].split("(")[0][:50]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg.setdefault(n, [0, 0.0]); agg[n][0] += 1; agg[n][1] += d
print("span us", (int(rows[z]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3, "kernels", z - a)
for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:25]:
    print(f"{d:9.1f} us  x{c:3d}  {n}")
PY
