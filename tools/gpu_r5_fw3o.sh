# round 5: the fused direct eigensolver at 3 workgroups per CU (no Cholesky overlap, 2-chunk ring, 168 VGPRs with
# spills: variants/fw3o) vs production (overlap, 3-chunk ring, 2 workgroups per CU): C2, two lanes and solo
OUT=gpurun_out/fw3o
mkdir -p $OUT
export TMPDIR=/tmp
c2() { name=$1; shift; env "$@" timeout -k 10 200 python3 -u tools/bench_configs.py --configs c2 --reps 5 > $OUT/$name.jsonl 2> $OUT/$name.err || { echo "$name rc=$?"; tail -5 $OUT/$name.err; return 1; }
python3 -c "import json; d=json.loads(open('$OUT/$name.jsonl').readline()); print('$name', d['value'], d['ms_per_job'], d['kernels_ms_per_job'], d.get('roofline_eig_fused',{}).get('frac'))"; }
for r in 1 2; do c2 prod_$r DFM_X=0 && c2 fw3o_$r DFM_LIB_PATH=variants/fw3o/libdfm.so || exit 1; done
c2 prod_solo DFM_NO_LANES=1 && c2 fw3o_solo DFM_NO_LANES=1 DFM_LIB_PATH=variants/fw3o/libdfm.so
