#!/bin/bash
# Round-end measurement session: the -m gpu suite, the headline bench line and
# the rocprofv3 summary of the same command, the config lines, and the C2
# kernel summary.  Each step bounded; stop at the first failure.
OUT=${1:-gpurun_out/fin}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { echo "pytest rc=$?"; tail -20 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
tools/gpu_bench_trace.sh "$OUT/bt" || exit 1
timeout -k 10 400 python3 -u tools/bench_configs.py --configs c1,c2,c4,c5 --reps 3 > "$OUT/configs.jsonl" 2> "$OUT/configs.err" || { echo "configs rc=$?"; tail -5 "$OUT/configs.err"; exit 1; }
cut -c1-160 "$OUT/configs.jsonl"
tools/gpu_c2_trace.sh "$OUT/c2" || exit 1
