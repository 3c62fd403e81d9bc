#!/bin/bash
# C3 bench kernel trace (rocprofv3 stats) + one bench line.
OUT=${1:-gpurun_out/g}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/trace.out" 2> "$OUT/trace.err" || { echo trace rc=$?; tail -20 "$OUT/trace.err"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/trace/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{r['Name'][:60]:60s} {int(r['Calls']):5d} {float(r['TotalDurationNs'])/1e6:8.2f} ms {float(r['AverageNs'])/1e3:8.1f} us")
PY
