# round 5: the default bench line, then the rocprofv3 kernel-trace summary of the same command
# (profiles/r05_bench.json, profiles/r05_bench_kernel_stats.csv)
OUT=gpurun_out/r5b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
cut -c1-400 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-all-fields > $OUT/bench_prof.json 2> $OUT/bench_prof.err; echo prof=$?
find $OUT/prof -name "*kernel_stats.csv" | head -3
