#!/bin/bash
# Shard-size sweep (the per-rank share of 9999 at N = 2/4/8) and a rocprofv3
# kernel trace of the 1250-replicate shard.  Exit other than 0/1 stops.
OUT=${1:-gpurun_out/shard}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 "$OUT/$name.err"; exit $rc; fi
  return 0
}
for R in 9999 5000 2500 1250; do
  step b$R 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --replicates $R
  python3 -c "import json,sys; d=json.loads(open('$OUT/b$R.out').read().strip().splitlines()[-1]); print($R, d['ms_per_step'], d['value'], d['eig_iterations'])"
done
step t1250 200 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/t1250" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --replicates 1250
echo ALLDONE
