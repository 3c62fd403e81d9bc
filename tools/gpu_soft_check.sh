#!/bin/bash
# Lasso session: the soft tests (bit-identity with the elnet1 restatement,
# clean launch records), the C4 line and the leaders' phase profile.
OUT=${1:-gpurun_out/soft}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_soft.py -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -4 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python3 -u tools/bench_configs.py --configs c4 --reps 5 > "$OUT/c4.jsonl" 2> "$OUT/c4.err" || { echo "c4 rc=$?"; tail -5 "$OUT/c4.err"; exit 1; }
cut -c1-600 "$OUT/c4.jsonl"
DFM_LASSO_PROF=1 timeout -k 10 300 python3 -u tools/bench_configs.py --configs c4 --reps 1 > "$OUT/c4p.jsonl" 2> "$OUT/c4p.err" || { echo "c4 prof rc=$?"; tail -5 "$OUT/c4p.err"; exit 1; }
tail -14 "$OUT/c4p.err"
