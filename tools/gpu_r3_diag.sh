#!/bin/bash
# Round-3 session: the -m gpu suite (no -x), then the exit-time SIGSEGV
# diagnosis: a bare cooperative launch under rocprofv3 (plain launch first),
# then C4 under rocprofv3 with /proc/self/maps dumped at exit.  Any exit other
# than 0/1 stops the session.
OUT=${1:-gpurun_out/diag}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {   # name, timeout, command...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 "$OUT/$name.err"; exit $rc; fi
  return 0
}
if [ -z "$SKIP_TESTS" ]; then
  step pytest 900 python -u -m pytest tests -m gpu -q --maxfail=200 --timeout 180 --timeout-method thread -p no:cacheprovider
  tail -5 "$OUT/pytest.out"
fi
step probe_plain 60 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/probe_plain" -o run -- ./tools/coop_exit_probe 1
cat "$OUT/probe_plain.out"
step probe_coop 60 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/probe_coop" -o run -- ./tools/coop_exit_probe 0
cat "$OUT/probe_coop.out"
step trace_c4 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace_c4" -o run -- python3 tools/bench_configs.py --configs c4 --reps 1 --dump-maps "$OUT/c4_maps.txt"
echo ALLDONE
