set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for sub in base replicas all; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$sub -o run -- python3 scripts/probe_single.py 5 $sub > gpurun_out/prof_$sub.log 2>&1 || exit 1
  rm -f gpurun_out/prof_$sub/run_kernel_trace.csv
  echo "== $sub"; grep -E "wall|updates|decode" gpurun_out/prof_$sub.log | head -3
  python3 - "$sub" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/prof_{sys.argv[1]}/run_kernel_stats.csv")))
for r in rows[:8]:
    print("%-50s %5s %9.1f us" % (r['Name'][:50], r['Calls'], float(r['AverageNs']) / 1e3))
PY
done
