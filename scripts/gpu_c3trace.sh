#!/bin/bash
# C3 kernel trace (per-dispatch durations of one merge)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
YCRDT_DEBUG_DECODE=1 timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c3trace -o c4 -- python3 scripts/probe_c3.py 10000000 256 16 > gpurun_out/c3trace.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/c3trace/**/*kernel_trace.csv", recursive=True)[0]
r = sorted(csv.DictReader(open(f)), key=lambda x: int(x["Start_Timestamp"]))
sp = [i for i, x in enumerate(r) if "k_spec" in x["Kernel_Name"]]
a = sp[-1]
out = open("gpurun_out/c3trace_last.txt", "w")
for x in r[a:a + 400]:
    s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
    out.write("%10.1f %8.1f %s\n" % ((s - int(r[a]["Start_Timestamp"])) / 1e3, (e - s) / 1e3, x["Kernel_Name"][:70]))
out.close()
PY
grep -E "k_spec|k_sync|k_walk|k_fastwalk|k_fastmark|k_chunk_counts|k_xtab|k_xmark|k_ds_decode|k_direct|k_wlen|k_wrank" gpurun_out/c3trace_last.txt | head -30
rm -rf gpurun_out/c3trace
grep "ycrdt decode" gpurun_out/c3trace.log | sort | uniq -c | head
