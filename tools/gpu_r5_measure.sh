# round 5 measurement session: C3 shard sizes, the other configs, PMC traffic of the H.Z GEMM
OUT=gpurun_out/r5m
mkdir -p $OUT
export TMPDIR=/tmp
for n in 1250 2500 5000 9999; do
  timeout -k 10 200 python3 -u bench.py --replicates $n --steps 20 --warmup 3 --no-cpu-baseline --no-all-fields > $OUT/s$n.json 2> $OUT/s$n.err || { echo "s$n rc=$?"; tail -5 $OUT/s$n.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print($n, d['value'], d['ms_per_step'])" $OUT/s$n.json
done
timeout -k 10 400 python3 -u tools/bench_configs.py --configs c1,c2,c4,c5 --reps 5 > $OUT/configs.jsonl 2> $OUT/configs.err || { echo "configs rc=$?"; tail -5 $OUT/configs.err; exit 1; }
cut -c1-600 $OUT/configs.jsonl
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gemmh_kernel|boot_" -f csv -d $OUT/pmc_f -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-all-fields > $OUT/pmc_f.out 2> $OUT/pmc_f.err; echo pmc_f=$?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gemmh_kernel|boot_" -f csv -d $OUT/pmc_w -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-all-fields > $OUT/pmc_w.out 2> $OUT/pmc_w.err; echo pmc_w=$?
python3 tools/pmc_traffic.py $OUT/pmc_f $OUT/pmc_w > $OUT/pmc_traffic.json && head -c 1500 $OUT/pmc_traffic.json
