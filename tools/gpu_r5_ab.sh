# round 5: production build vs a variant library ($VAR, tag $TAG): C3 headline and its 1250 shard, alternating
# (and C2 when $C2=1); then the GPU suite
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
b() { name=$1; lib=$2; shift 2; if [ "$lib" = "-" ]; then unset DFM_LIB_PATH; else export DFM_LIB_PATH=$lib; fi
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-all-fields "$@" > $OUT/$name.json 2> $OUT/$name.err || { echo "$name rc=$?"; tail -5 $OUT/$name.err; return 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], d['kernels_ms'], [(h['kernel'][:14], h['frac']) for h in d.get('roofline_hbm', [])], d['roofline']['frac'])" $OUT/$name.json; }
c2() { name=$1; lib=$2; if [ "$lib" = "-" ]; then unset DFM_LIB_PATH; else export DFM_LIB_PATH=$lib; fi
  timeout -k 10 200 python3 -u tools/bench_configs.py --configs c2 --reps 5 > $OUT/$name.jsonl 2> $OUT/$name.err || { echo "$name rc=$?"; tail -5 $OUT/$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$name.jsonl').readline()); print('$name', d['value'], d['ms_per_job'], d['kernels_ms_per_job'])"; }
for r in 1 2; do
  b new_$r - --steps 20 --warmup 3 && b var_$r $VAR --steps 20 --warmup 3 || exit 1
  b new1250_$r - --replicates 1250 --steps 20 --warmup 3 && b var1250_$r $VAR --replicates 1250 --steps 20 --warmup 3 || exit 1
  if [ "$C2" = 1 ]; then c2 newc2_$r - && c2 varc2_$r $VAR || exit 1; fi
done
unset DFM_LIB_PATH
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.txt 2>&1; echo pytest_rc=$?; tail -3 $OUT/pytest.txt
