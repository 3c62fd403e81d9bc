# round 5 close (after the host-turnaround work): default bench line + its rocprofv3 kernel summary, the shard sizes,
# the config lines, C5 panel-resident windows, then the GPU suite -> profiles/r05_*
OUT=gpurun_out/r5c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-all-fields > $OUT/bench_prof.json 2> $OUT/bench_prof.err; echo prof=$?
for n in 1250 2500 5000 9999; do
  timeout -k 10 200 python3 -u bench.py --replicates $n --steps 20 --warmup 3 --no-cpu-baseline --no-all-fields > $OUT/s$n.json 2> $OUT/s$n.err || { echo "s$n rc=$?"; tail -5 $OUT/s$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print($n, d['value'], d['ms_per_step'])" $OUT/s$n.json
done
timeout -k 10 400 python3 -u tools/bench_configs.py --configs c1,c2,c4,c5 --reps 5 > $OUT/configs.jsonl 2> $OUT/configs.err || { echo "configs rc=$?"; tail -5 $OUT/configs.err; exit 1; }
cut -c1-300 $OUT/configs.jsonl
for L in 0 1000; do
  timeout -k 10 300 python3 -u bench.py --workload c5 --rolling $L --no-cpu-baseline > $OUT/c5_$L.json 2> $OUT/c5_$L.err || { echo "c5 rc=$?"; tail -5 $OUT/c5_$L.err; exit 1; }
  cut -c1-200 $OUT/c5_$L.json
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $OUT/pytest.txt 2>&1; echo pytest_rc=$?; tail -3 $OUT/pytest.txt
