#!/bin/bash
# The headline bench line and the rocprofv3 kernel summary of the same
# (default) command.
OUT=${1:-gpurun_out/bt}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench rc=$?"; tail -5 "$OUT/bench.err"; exit 1; }
tail -1 "$OUT/bench.json" | cut -c1-1200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/trace.out" 2> "$OUT/trace.err" || { echo "trace rc=$?"; tail -5 "$OUT/trace.err"; exit 1; }
head -3 "$OUT/trace/run_kernel_stats.csv" | cut -c1-200
