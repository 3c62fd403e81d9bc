#!/bin/bash
# Round-3 session C: eigensolver size scaling, the failing GPU tests, and the
# HZ non-temporal-store A/B.  Exit other than 0/1 stops.
OUT=${1:-gpurun_out/c}
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
step pytest 600 python -u -m pytest tests/test_gpu_breaks.py tests/test_gpu_windows_ex.py tests/test_gpu_spectrum.py tests/test_gpu_parity.py -m gpu -v -rf --maxfail=50 --timeout 300 --timeout-method thread -p no:cacheprovider -k "not beyond_factored"
grep -E "FAILED|passed|failed" "$OUT/pytest.out" | tail -20
step ab 600 bash tools/ab_bench.sh "$OUT/ab" 3 "base|-|--steps 10 --warmup 3" "hznt|variants/hz_nt/libdfm.so|--steps 10 --warmup 3"
cat "$OUT/ab.out"
step eigscale 150 python -u tools/eig_scale_probe.py 512 1024 2048 3072 4000
cat "$OUT/eigscale.out"
echo ALLDONE
