#!/bin/bash
# Headline (C3) bench A/B over variant libraries (DFM_LIB_PATH), alternating.
#   tools/gpu_c3_ab.sh OUTDIR ROUNDS name=libpath ...   ("-" = production)
OUT=$1; ROUNDS=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 "$ROUNDS"); do
  for spec in "$@"; do
    name=${spec%%=*}; lib=${spec#*=}
    if [ "$lib" = "-" ]; then unset DFM_LIB_PATH; else export DFM_LIB_PATH="$lib"; fi
    timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/c3_${name}_$r.json" 2> "$OUT/c3_${name}_$r.err"
    rc=$?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c3', sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" "$OUT/c3_${name}_$r.json" "$name" "$r" 2>/dev/null || echo "c3 $name $r rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/c3_${name}_$r.err"; exit $rc; fi
  done
done
unset DFM_LIB_PATH
