#!/bin/bash
# The -m gpu suite (stop on the first failure), then another GPU script.
# Usage: tools/gpu_tests_then.sh OUTDIR script [args...]
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -6 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
"$@"
