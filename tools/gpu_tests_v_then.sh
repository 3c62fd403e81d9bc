#!/bin/bash
# The -m gpu suite verbose (the log lists every test), then another GPU script.
# Usage: tools/gpu_tests_v_then.sh OUTDIR script [args...]
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 180 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then grep -n "FAILED\|Error" "$OUT/pytest.log" | head; echo "pytest rc=$rc: stopping"; exit $rc; fi
"$@"
