#!/bin/bash
# Two-lane small-job bootstrap + soft Grams on the DMA path: the affected GPU
# tests, then shard-size timings and C4.  Exit other than 0/1 stops.
OUT=${1:-gpurun_out/lane}
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
step pytest 400 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_breaks.py tests/test_gpu_compaction.py tests/test_gpu_production.py tests/test_gpu_parity.py tests/test_gpu_soft.py -q --maxfail=10 --timeout 200 --timeout-method thread -p no:cacheprovider
tail -5 "$OUT/pytest.out"
for R in 1250 2500 5000 9999; do
  step b$R 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --replicates $R
  python3 -c "import json,sys; d=json.loads(open('$OUT/b$R.out').read().strip().splitlines()[-1]); print($R, d['ms_per_step'], d['value'], d['roofline']['frac'], d['eig_iterations'])"
done
step c4 300 python -u tools/bench_configs.py --configs c2,c4 --reps 3
tail -2 "$OUT/c4.out"
step trace_c4 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace_c4" -o run -- python3 tools/bench_configs.py --configs c4 --reps 1
echo ALLDONE
