# round 5: DRAM traffic per launch of the C2 job's kernels (FETCH_SIZE and WRITE_SIZE in separate passes)
OUT=gpurun_out/pmc_c2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/f -o run -- python3 tools/bench_configs.py --configs c2 --reps 1 > $OUT/f.out 2> $OUT/f.err; echo f=$?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/w -o run -- python3 tools/bench_configs.py --configs c2 --reps 1 > $OUT/w.out 2> $OUT/w.err; echo w=$?
python3 tools/pmc_traffic.py $OUT/f $OUT/w > $OUT/pmc_traffic_c2.json && python3 -c "import json; d=json.load(open('$OUT/pmc_traffic_c2.json')); [print(k[:40], round(v['hbm_bytes_per_launch']/1e6,2), 'MB', v['launches_fetch_pass']) for k,v in d.items()]"
