# round 5: the fused direct eigensolver's products on v_mfma_f64_16x16x4 (production build, 2 waves/SIMD),
# the same at 3 waves/SIMD (variants/fw3) and the previous 4x4x4_4b form (variants/fz4): C2 A/B, then the GPU suite
OUT=gpurun_out/fz16
mkdir -p $OUT
export TMPDIR=/tmp
c2() { name=$1; shift; env "$@" timeout -k 10 200 python3 -u tools/bench_configs.py --configs c2 --reps 5 > $OUT/$name.jsonl 2> $OUT/$name.err || { echo "$name rc=$?"; tail -5 $OUT/$name.err; return 1; }
python3 -c "import json; d=json.loads(open('$OUT/$name.jsonl').readline()); print('$name', d['value'], d['ms_per_job'], d['kernels_ms_per_job'], d.get('roofline_eig_fused',{}).get('frac'))"; }
for r in 1 2; do
  c2 new_$r DFM_X=0 && c2 fw3_$r DFM_LIB_PATH=variants/fw3/libdfm.so && c2 fz4_$r DFM_LIB_PATH=variants/fz4/libdfm.so || exit 1
done
c2 new_solo DFM_NO_LANES=1 && c2 fw3_solo DFM_NO_LANES=1 DFM_LIB_PATH=variants/fw3/libdfm.so && c2 fz4_solo DFM_NO_LANES=1 DFM_LIB_PATH=variants/fz4/libdfm.so || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.txt 2>&1; echo pytest_rc=$?; tail -3 $OUT/pytest.txt
