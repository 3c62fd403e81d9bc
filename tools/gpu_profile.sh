#!/bin/bash
# One GPU session: parity tests, bench, kernel-trace stats, two PMC passes for
# HBM traffic of the dominant kernel.  Usage: tools/gpu_profile.sh OUTDIR [bench args]
set -o pipefail
OUT=${1:-gpurun_out/prof}; shift
BARGS="$@"
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u bench.py $BARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $BARGS > "$OUT/bench_trace.json" 2> "$OUT/trace.err" || { echo "trace failed"; tail -20 "$OUT/trace.err"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gemm|gram_kernel|gram_dma|boot_y2|boot_ap2|boot_cheb" -f csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline $BARGS > /dev/null 2> "$OUT/pmc_fetch.err" || { echo "pmc fetch failed"; tail -20 "$OUT/pmc_fetch.err"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gemm|gram_kernel|gram_dma|boot_y2|boot_ap2|boot_cheb" -f csv -d "$OUT/pmc_write" -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline $BARGS > /dev/null 2> "$OUT/pmc_write.err" || { echo "pmc write failed"; tail -20 "$OUT/pmc_write.err"; exit 1; }
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" > "$OUT/pmc_traffic.json"
cat "$OUT/pmc_traffic.json"
echo ALLDONE
