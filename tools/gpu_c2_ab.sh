#!/bin/bash
# C2 config line A/B over variant libraries (DFM_LIB_PATH), alternating.
#   tools/gpu_c2_ab.sh OUTDIR ROUNDS name=libpath ...   ("-" = production)
OUT=$1; ROUNDS=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 "$ROUNDS"); do
  for spec in "$@"; do
    name=${spec%%=*}; lib=${spec#*=}
    if [ "$lib" = "-" ]; then unset DFM_LIB_PATH; else export DFM_LIB_PATH="$lib"; fi
    timeout -k 10 200 python3 -u tools/bench_configs.py --configs c2 --reps 5 > "$OUT/${name}_$r.jsonl" 2> "$OUT/${name}_$r.err"
    rc=$?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_job'], d['kernels_ms_per_job'].get('chow'))" "$OUT/${name}_$r.jsonl" "$name" "$r" 2>/dev/null || echo "$name $r rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/${name}_$r.err"; exit $rc; fi
  done
done
unset DFM_LIB_PATH
