#!/bin/bash
# Full GPU suite, shard timings, C2 and its kernel trace.  Exit other than 0/1 stops.
OUT=${1:-gpurun_out/f}
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
step pytest 600 python -u -m pytest tests -m gpu -v --maxfail=20 --timeout 100 --timeout-method thread -p no:cacheprovider
tail -4 "$OUT/pytest.out"
for R in 1250 2500 9999; do
  step b$R 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --replicates $R
  python3 -c "import json,sys; d=json.loads(open('$OUT/b$R.out').read().strip().splitlines()[-1]); print($R, d['ms_per_step'], d['value'], d['roofline']['frac'], d['eig_iterations'])"
done
step c2 300 python -u tools/bench_configs.py --configs c1,c2 --reps 3
tail -2 "$OUT/c2.out"
step trace_c2 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace_c2" -o run -- python3 tools/bench_configs.py --configs c2 --reps 2
echo ALLDONE
