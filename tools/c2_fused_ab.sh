OUT=gpurun_out/r06o; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do
for v in prod f1; do
  if [ $v = prod ]; then unset DFM_LIB_PATH; else export DFM_LIB_PATH=abv/f1/libdfm.so; fi
  timeout -k 10 200 python3 -u tools/bench_configs.py --configs c2 --reps 5 > $OUT/${v}_$r.jsonl 2> $OUT/${v}_$r.err || { echo "$v rc=$?"; tail -5 $OUT/${v}_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_job'], d['kernels_ms_per_job'])" $OUT/${v}_$r.jsonl $v
  DFM_NO_LANES=1 DFM_EIG_PROF=1 timeout -k 10 200 python3 -u tools/bench_configs.py --configs c2 --reps 2 > $OUT/${v}_solo_$r.jsonl 2> $OUT/${v}_solo_$r.err || { echo "$v solo rc=$?"; tail -5 $OUT/${v}_solo_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], 'solo', d['value'], d['ms_per_job'], d['kernels_ms_per_job'])" $OUT/${v}_solo_$r.jsonl $v
  grep "eig_fused m=" $OUT/${v}_solo_$r.err | tail -2
done
done
