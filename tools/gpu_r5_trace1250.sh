# round 5: kernel + HIP API trace of the 1250-replicate C3 shard (where the host turnaround goes between and inside steps)
OUT=gpurun_out/tr1250
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -f csv -d $OUT/prof -o run -- python3 bench.py --replicates 1250 --steps 10 --warmup 3 --no-cpu-baseline --no-all-fields > $OUT/bench.json 2> $OUT/bench.err
echo rc=$?
find $OUT -name "*.csv" | head
