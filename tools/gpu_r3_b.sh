#!/bin/bash
# Round-3 session B: big-T window probe, the -m gpu suite (verbose, one known-slow
# case deselected), the C3 iteration histogram, C4 under rocprofv3 (the lasso's
# plain co-resident launch), the headline bench.  Exit other than 0/1 stops.
OUT=${1:-gpurun_out/b}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {   # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 "$OUT/$name.err"; exit $rc; fi
  return 0
}
step pytest 1500 python -u -m pytest tests -m gpu -v -rf --maxfail=200 --timeout 300 --timeout-method thread -p no:cacheprovider -k "not beyond_factored"
grep -E "FAILED|passed|failed" "$OUT/pytest.out" | tail -40
step iters 200 python -u tools/c3_iters.py 2000
cat "$OUT/iters.out"
step trace_c4 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace_c4" -o run -- python3 tools/bench_configs.py --configs c4 --reps 1
cat "$OUT/trace_c4.out"
step bench 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 5
cat "$OUT/bench.out"
step bigT_pca 100 python -u tools/windows_bigT_probe.py pca 4200
cat "$OUT/bigT_pca.out"
step bigT_win 100 python -u tools/windows_bigT_probe.py windows 4200
cat "$OUT/bigT_win.out"
echo ALLDONE
