# round 5: C2 (two lanes) with the second lane held back on the device (variants/skew, DFM_LANE_SKEW_US), alternating
OUT=gpurun_out/skew
mkdir -p $OUT
export TMPDIR=/tmp
c2() { name=$1; timeout -k 10 200 python3 -u tools/bench_configs.py --configs c2 --reps 5 > $OUT/$name.jsonl 2> $OUT/$name.err || { echo "$name rc=$?"; tail -5 $OUT/$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$name.jsonl').readline()); print('$name', d['value'], d['ms_per_job'])"; }
for r in 1 2; do
  unset DFM_LIB_PATH DFM_LANE_SKEW_US; c2 prod_$r || exit 1
  export DFM_LIB_PATH=variants/skew/libdfm.so
  for us in 150 300 450 600; do DFM_LANE_SKEW_US=$us c2 skew${us}_$r || exit 1; done
done
