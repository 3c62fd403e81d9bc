#!/bin/bash
# A/B timing of the headline bench: alternating runs of named configurations
# (a variant library through DFM_LIB_PATH and/or extra bench.py flags).
#   tools/ab_bench.sh OUTDIR ROUNDS "name|libpath|flags" ...
# libpath "-" = the production library.  Each run has its own time limit; a
# run that faults or times out ends the session.
OUT=$1; ROUNDS=$2; shift 2
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for spec in "$@"; do
    IFS='|' read -r name lib flags <<< "$spec"
    if [ "$lib" = "-" ]; then unset DFM_LIB_PATH; else export DFM_LIB_PATH="$lib"; fi
    timeout -k 10 180 python -u bench.py --no-cpu-baseline $flags > "$OUT/${name}_$r.json" 2> "$OUT/${name}_$r.err"
    rc=$?
    python3 -c "import json,sys; d=json.loads(open('$OUT/${name}_$r.json').read().strip().splitlines()[-1]); print('$name', $r, d['ms_per_step'], d['value'], d['roofline']['frac'] if d.get('roofline') else None, d.get('eig_iterations'))" 2>/dev/null || echo "$name $r rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/${name}_$r.err"; exit $rc; fi
  done
done
unset DFM_LIB_PATH
