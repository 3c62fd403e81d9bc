#!/bin/bash
# Round measurement session: -m gpu suite, the headline bench, rocprofv3
# kernel stats of the bench (C3 factored) and of the direct-Gram mode and C2,
# then the PMC HBM-traffic passes.  Every GPU step has its own time limit; a
# fault / abort / timeout stops the session.
OUT=${1:-gpurun_out/measure}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {   # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -20 "$OUT/$name.err"; exit $rc; fi
  return 0
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest 900 python -u -m pytest tests -m gpu -v --maxfail=20 --timeout 100 --timeout-method thread -p no:cacheprovider
  tail -8 "$OUT/pytest.out"
fi
step bench 300 python -u bench.py --steps 20 --warmup 5
cat "$OUT/bench.out"
step trace 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
step bench_direct 300 python -u bench.py --steps 3 --warmup 1 --mode direct --no-cpu-baseline
step trace_direct 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace_direct" -o run -- python3 bench.py --steps 2 --warmup 1 --mode direct --no-cpu-baseline
step configs 600 python -u tools/bench_configs.py --configs c1,c2,c4,c5 --reps 3
cat "$OUT/configs.out"
step trace_c2 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace_c2" -o run -- python3 tools/bench_configs.py --configs c2 --reps 2
step trace_c4 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace_c4" -o run -- python3 tools/bench_configs.py --configs c4 --reps 1
step c5 300 python -u bench.py --workload c5 --steps 10 --warmup 2 --no-cpu-baseline
tail -1 "$OUT/c5.out"
step c5_rolling 300 python -u bench.py --workload c5 --rolling 1000 --steps 10 --warmup 2 --no-cpu-baseline
tail -1 "$OUT/c5_rolling.out"
for R in 5000 2500 1250; do   # the per-rank share of the 9999 replicates at N = 2 / 4 / 8
  step shard$R 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --replicates $R
  tail -1 "$OUT/shard$R.out"
done
step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gemm|gram_kernel|gram_dma|boot_|chow" -f csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
step pmc_write 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gemm|gram_kernel|gram_dma|boot_|chow" -f csv -d "$OUT/pmc_write" -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" > "$OUT/pmc_traffic.json"
# C2's Chow / Gram / eigen kernels (the bench passes above never launch them)
step pmc_fetch_c2 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "chow|gram_wk|gemmh|eig_|factors" -f csv -d "$OUT/pmc_fetch_c2" -o run -- python3 tools/bench_configs.py --configs c2 --reps 1
step pmc_write_c2 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "chow|gram_wk|gemmh|eig_|factors" -f csv -d "$OUT/pmc_write_c2" -o run -- python3 tools/bench_configs.py --configs c2 --reps 1
python3 tools/pmc_traffic.py "$OUT/pmc_fetch_c2" "$OUT/pmc_write_c2" > "$OUT/pmc_traffic_c2.json"
echo ALLDONE
