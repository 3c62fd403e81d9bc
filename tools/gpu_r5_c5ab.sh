# round 5: C5 windows (panel resident, expanding and rolling 1000) with the production library vs $VAR, alternating
OUT=gpurun_out/c5ab
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in new:- var:$VAR; do
    n=${v%%:*}; l=${v#*:}
    if [ "$l" = "-" ]; then unset DFM_LIB_PATH; else export DFM_LIB_PATH=$l; fi
    for L in 0 1000; do
      timeout -k 10 300 python3 -u bench.py --workload c5 --rolling $L --no-cpu-baseline --steps 10 --warmup 2 > $OUT/${n}_${L}_$r.json 2> $OUT/${n}_${L}_$r.err || { echo "$n rc=$?"; tail -5 $OUT/${n}_${L}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$n', $L, $r, d['value'], d['ms_per_step'])" $OUT/${n}_${L}_$r.json
    done
  done
done
