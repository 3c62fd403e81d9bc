# round 5: kernel + HIP API trace of the C2 job (two lanes): GPU idle time and the host calls around it
OUT=gpurun_out/trc2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -f csv -d $OUT/prof -o run -- python3 tools/bench_configs.py --configs c2 --reps 5 > $OUT/c2.jsonl 2> $OUT/c2.err
echo rc=$?
