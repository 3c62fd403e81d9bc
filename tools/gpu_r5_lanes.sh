# round 5: lanes per small bootstrap job (DFM_LANES A/B): C3 shards of 1250 / 2500 replicates, C2 (999)
OUT=gpurun_out/r5l
mkdir -p $OUT
export TMPDIR=/tmp
for round in 1 2; do
  for n in 2 3 4; do
    for B in 1250 2500; do
      DFM_LANES=$n timeout -k 10 200 python3 -u bench.py --replicates $B --steps 20 --warmup 3 --no-cpu-baseline --no-all-fields > $OUT/s${B}_l$n.json 2> $OUT/s${B}_l$n.err || { echo "s$B l$n rc=$?"; tail -5 $OUT/s${B}_l$n.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print('round $round lanes $n B $B', d['value'], d['ms_per_step'])" $OUT/s${B}_l$n.json
    done
    DFM_LANES=$n timeout -k 10 200 python3 -u tools/bench_configs.py --configs c2 --reps 5 > $OUT/c2_l$n.jsonl 2> $OUT/c2_l$n.err || { echo "c2 l$n rc=$?"; tail -5 $OUT/c2_l$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c2_l$n.jsonl').readline()); print('round $round lanes $n c2', d['value'], d['ms_per_job'])"
  done
done
