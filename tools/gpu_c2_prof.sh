#!/bin/bash
# C2 config line with the fused solver's phase profile (DFM_EIG_PROF=1 -> stderr).
OUT=${1:-gpurun_out/c2p}
mkdir -p "$OUT"
export TMPDIR=/tmp
DFM_EIG_PROF=1 timeout -k 10 300 python3 -u tools/bench_configs.py --configs c2 --reps 2 > "$OUT/c2_prof.jsonl" 2> "$OUT/c2_prof.err" || { echo "c2 prof rc=$?"; tail -5 "$OUT/c2_prof.err"; exit 1; }
grep eig_fused "$OUT/c2_prof.err" | tail -8
timeout -k 10 300 python3 -u tools/bench_configs.py --configs c2 --reps 5 > "$OUT/c2.jsonl" 2> "$OUT/c2.err" || { echo "c2 rc=$?"; tail -5 "$OUT/c2.err"; exit 1; }
cut -c1-330 "$OUT/c2.jsonl"
