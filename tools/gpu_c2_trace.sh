#!/bin/bash
# rocprofv3 kernel summary of the C2 config line (3 jobs).
OUT=${1:-gpurun_out/c2t}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$NOLANES" ]; then export DFM_NO_LANES=1; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/c2trace" -o run -- python3 tools/bench_configs.py --configs c2 --reps 3 > "$OUT/c2trace.out" 2> "$OUT/c2trace.err" || { echo "c2 trace rc=$?"; tail -5 "$OUT/c2trace.err"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/c2trace/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:18]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['TotalDurationNs'])/1e6:8.2f} ms {float(r['AverageNs'])/1e3:8.1f} us")
PY
