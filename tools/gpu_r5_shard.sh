# round 5: where a 1250-replicate C3 shard (one GPU of eight) spends its time: two lanes vs one, kernel summaries
# (profiles/r05_shard1250_*.csv)
OUT=gpurun_out/r5s
mkdir -p $OUT
export TMPDIR=/tmp
for v in lanes nolanes; do
  if [ $v = nolanes ]; then export DFM_NO_LANES=1; else unset DFM_NO_LANES; fi
  timeout -k 10 200 python3 -u bench.py --replicates 1250 --steps 20 --warmup 3 --no-cpu-baseline --no-all-fields > $OUT/$v.json 2> $OUT/$v.err || { echo "$v rc=$?"; tail -5 $OUT/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('$v', d['value'], d['ms_per_step'], d['kernels_ms'], d['eig_iterations'])" $OUT/$v.json
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$v -o run -- python3 bench.py --replicates 1250 --steps 20 --warmup 3 --no-cpu-baseline --no-all-fields > $OUT/prof_$v.json 2> $OUT/prof_$v.err; echo prof_$v=$?
done
unset DFM_NO_LANES
