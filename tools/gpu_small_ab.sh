#!/bin/bash
# Rayleigh-Ritz step variants on C2: Jacobi sweeps 2 / 1, chol(Z'Z) vs column norms.
OUT=${1:-gpurun_out/sab}
mkdir -p "$OUT"
export TMPDIR=/tmp
for V in "2 0" "1 0" "2 1" "1 1"; do
  set -- $V
  DFM_EIG_JSWEEPS=$1 DFM_EIG_DIAGNORM=$2 DFM_EIG_PROF=1 timeout -k 10 300 python3 -u tools/bench_configs.py --configs c2 --reps 5 > "$OUT/c2_$1_$2.jsonl" 2> "$OUT/c2_$1_$2.err" || { echo "c2 $V rc=$?"; tail -5 "$OUT/c2_$1_$2.err"; exit 1; }
  echo "== sweeps=$1 diagnorm=$2"
  grep eig_fused "$OUT/c2_$1_$2.err" | tail -2
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(d['value'], d['ms_per_job'], d['eig_iterations'])" "$OUT/c2_$1_$2.jsonl"
done
