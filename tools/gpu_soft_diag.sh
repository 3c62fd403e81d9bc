#!/bin/bash
# Lasso hand-off diagnosis: many back-to-back soft selections with a short
# spin timeout (every timed-out spin is described on stderr by the launch
# record), then the soft GPU tests at the production timeout.
OUT=${1:-gpurun_out/softdiag}
N=${2:-1000}
mkdir -p "$OUT"
export TMPDIR=/tmp
DFM_LASSO_TMO_MS=${TMO_MS:-50} timeout -k 10 400 python3 -u tools/soft_repeat.py "$N" > "$OUT/rep.out" 2> "$OUT/rep.err"
rc=$?
tail -8 "$OUT/rep.out"; grep -c "timed out" "$OUT/rep.err"; grep "timed out" "$OUT/rep.err" | head -20
if [ $rc -ne 0 ]; then echo "repeat rc=$rc"; exit $rc; fi
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_soft.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -15 "$OUT/pytest.log"
echo "pytest rc=$rc"
