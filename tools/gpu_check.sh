#!/bin/bash
# One GPU session: the -m gpu suite (no -x: every failure listed), then a short
# bench.  A test-runner exit of 0/1 (pass / test failures) continues to the
# bench; anything else (fault, abort, timeout) stops the session.
# Usage: [KEXPR="not slow"] tools/gpu_check.sh OUTDIR [pytest selection]
OUT=${1:-gpurun_out/check}; shift
SEL=${@:-tests}
mkdir -p "$OUT"
export TMPDIR=/tmp
KARGS=()
[ -n "$KEXPR" ] && KARGS=(-k "$KEXPR")
timeout -k 10 900 python -u -m pytest $SEL "${KARGS[@]}" -m gpu -q --maxfail=15 --timeout 180 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -25 "$OUT/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 6 > "$OUT/bench.json" 2> "$OUT/bench.err"
brc=$?
cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"
echo "pytest rc=$rc bench rc=$brc"
