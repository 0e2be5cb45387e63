set -u
mkdir -p gpurun_out/hl
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/hl -o hl -- python3 bench.py --only-headline --steps 3 --warmup 1 > gpurun_out/hl/bench.json 2> gpurun_out/hl/bench.err || { tail -20 gpurun_out/hl/bench.err; exit 1; }
python3 scripts/bench_summary.py gpurun_out/hl/bench.json
f=$(find gpurun_out/hl -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dec = [i for i, r in enumerate(rows) if "k_struct_decode(" in r["Kernel_Name"] or "k_struct_decode<" in r["Kernel_Name"]]
a, z = dec[-2], dec[-1]
# one merge: from the kernel after the previous merge's last write to this one: take the window between two struct decodes
cnt = collections.Counter(r["Kernel_Name"].split("(")[0][:60] for r in rows[a:z])
print("dispatches between two struct decodes:", z - a)
for n, c in cnt.most_common(60):
    print(f"{c:3d} {n}")
PY
