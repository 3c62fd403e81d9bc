#!/bin/bash
# C3 shard of 1250 replicates (the 8-GPU per-rank share of B = 9999): bench
# line + rocprofv3 kernel summary; then the C4 config line.
OUT=${1:-gpurun_out/shard}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --replicates 1250 --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/s1250.json" 2> "$OUT/s1250.err" || { echo "s1250 rc=$?"; tail -5 "$OUT/s1250.err"; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(d['value'], d['ms_per_step'], d.get('kernels_ms'), d.get('kernel_launches'))" "$OUT/s1250.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 bench.py --replicates 1250 --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/trace.out" 2> "$OUT/trace.err" || { echo "trace rc=$?"; tail -5 "$OUT/trace.err"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/trace/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['TotalDurationNs'])/1e6:8.2f} ms {float(r['AverageNs'])/1e3:8.1f} us")
PY
timeout -k 10 300 python3 -u tools/bench_configs.py --configs c4 --reps 3 > "$OUT/c4.jsonl" 2> "$OUT/c4.err" || { echo "c4 rc=$?"; tail -5 "$OUT/c4.err"; exit 1; }
cut -c1-900 "$OUT/c4.jsonl"
