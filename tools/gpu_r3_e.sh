#!/bin/bash
# Round-3 session E: the whole GPU suite, the C2 accuracy probe with the
# subspace convergence rule (production: LM keeps F'E_i; variant: F'E_i
# assumed 0), C2 timing with the batched-gather Chow kernel, the C3 bench.
# Exit other than 0/1 stops.
OUT=${1:-gpurun_out/e}
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
step pytest 900 python -u -m pytest tests -m gpu -v -rf --maxfail=50 --timeout 300 --timeout-method thread -p no:cacheprovider
grep -E "FAILED|passed|failed" "$OUT/pytest.out" | tail -20
step c2tol 300 python -u tools/c2_tol_probe.py
cat "$OUT/c2tol.out"
DFM_LIB_PATH=variants/nocf/libdfm.so step c2tol_nocf 300 python -u tools/c2_tol_probe.py
cat "$OUT/c2tol_nocf.out"
step c2 200 python -u tools/bench_configs.py --configs c2 --reps 3
tail -1 "$OUT/c2.out"
step bench 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline
tail -1 "$OUT/bench.out"
echo ALLDONE
