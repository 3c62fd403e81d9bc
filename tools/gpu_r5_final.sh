# round 5 close: the default bench line, the rocprofv3 kernel summary of the same workload, the config lines
# (C2 with its eig_fused and Chow rooflines), then the GPU suite -> profiles/r05_final_*
OUT=gpurun_out/r5f
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench rc=$?"; tail -5 $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --no-cpu-baseline --no-all-fields > $OUT/bench_prof.json 2> $OUT/bench_prof.err; echo prof=$?
timeout -k 10 400 python3 -u tools/bench_configs.py --configs c1,c2,c4,c5 --reps 5 > $OUT/configs.jsonl 2> $OUT/configs.err || { echo "configs rc=$?"; tail -5 $OUT/configs.err; exit 1; }
cut -c1-300 $OUT/configs.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > $OUT/pytest.txt 2>&1; echo pytest_rc=$?; tail -3 $OUT/pytest.txt
