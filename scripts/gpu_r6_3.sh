set -u
mkdir -p gpurun_out/fs3
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/probe_small_large2.py 1 0 > gpurun_out/r6_sl4.log 2>&1; grep -A1 PREDECODE gpurun_out/r6_sl4.log; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fs3 -o fs -- python3 scripts/probe_fullstate.py nt:YCRDT_RTAB=0 > gpurun_out/fs3/probe.log 2>&1 || { tail -20 gpurun_out/fs3/probe.log; exit 1; }
grep -v "^W2026\|^E2026" gpurun_out/fs3/probe.log | grep "ms, device\|{\|equal"
f=$(find gpurun_out/fs3 -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
spec = [i for i, r in enumerate(rows) if "k_spec" in r["Kernel_Name"]]
# the third record-mode merge with the table (config "1": merges 1..4 of the run's k_spec list; take the 4th k_spec)
for label, k in (("table", 3), ("notable", 11)):
    if k + 1 >= len(spec): continue
    a, z = spec[k], spec[k + 1]
    agg = collections.OrderedDict()
    for r in rows[a - 3:z - 3]:
        n = r["Kernel_Name"].split("(")[0][:50]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        agg.setdefault(n, [0, 0.0]); agg[n][0] += 1; agg[n][1] += d
    print(label, " ".join(f"{n.replace('yc::','')}:{d:.0f}" for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:14]))
PY
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fastwalk.py tests/test_gpu_large_ds.py tests/test_gpu_chunk_path.py tests/test_gpu_decode_paths.py tests/test_gpu_ds_edges.py tests/test_gpu_predecode.py tests/test_gpu_edges.py > gpurun_out/r6_t3.log 2>&1
rc=$?; echo "[tests] rc=$rc"; tail -n 3 gpurun_out/r6_t3.log; [ $rc -eq 0 ] || { grep -n "FAILED\|Error\|assert" gpurun_out/r6_t3.log | head -30; exit $rc; }
