#!/bin/bash
# A selection of -m gpu tests in one process (each test bounded), log under OUT.
# Usage: tools/gpu_tests.sh OUT 'pytest selection ...' [-k expr]
OUT=${1:-gpurun_out/t}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest "$@" -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -40
echo "pytest rc=$rc"
exit $rc
