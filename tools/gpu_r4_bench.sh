#!/bin/bash
# Round-4 measurement session: C3 bench line, C2/C4 config lines, and the
# rocprofv3 kernel summary of the C2 job (each step bounded; stop on failure).
OUT=${1:-gpurun_out/r4b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/c3.json" 2> "$OUT/c3.err" || { echo "c3 rc=$?"; tail -5 "$OUT/c3.err"; exit 1; }
cat "$OUT/c3.json"
timeout -k 10 300 python3 -u tools/bench_configs.py --configs c2,c4 --reps 5 > "$OUT/configs.jsonl" 2> "$OUT/configs.err" || { echo "configs rc=$?"; tail -5 "$OUT/configs.err"; exit 1; }
cat "$OUT/configs.jsonl"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/c2trace" -o run -- python3 tools/bench_configs.py --configs c2 --reps 3 > "$OUT/c2trace.out" 2> "$OUT/c2trace.err" || { echo "c2 trace rc=$?"; tail -5 "$OUT/c2trace.err"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/c2trace/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['TotalDurationNs'])/1e6:8.2f} ms {float(r['AverageNs'])/1e3:8.1f} us")
PY
