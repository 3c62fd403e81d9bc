# round 5 (CHOW_VARS / CHOW_TEST / CHOW_OUT select other variant sets): the Chow kernel at exact R = 3 (variants/ch3: 3 waves per SIMD,
# variants/ch3w4: 4 waves) against the production R = 4 form: C2 job rate
# (two lanes) and solo kernel times (DFM_NO_LANES=1), alternating; then the
# Chow / C2 GPU tests on each variant
OUT=gpurun_out/${CHOW_OUT:-chow3}
mkdir -p $OUT
export TMPDIR=/tmp
c2() { name=$1; lib=$2; if [ "$lib" = "-" ]; then unset DFM_LIB_PATH; else export DFM_LIB_PATH=$lib; fi
  timeout -k 10 200 python3 -u tools/bench_configs.py --configs c2 --reps 5 > $OUT/$name.jsonl 2> $OUT/$name.err || { echo "$name rc=$?"; tail -5 $OUT/$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$name.jsonl').readline()); print('$name', d['value'], d['ms_per_job'], d['kernels_ms_per_job'], d.get('roofline_chow', {}).get('frac'))"; }
for r in 1 2; do
  for v in ${CHOW_VARS:-prod:- ch3:variants/ch3/libdfm.so ch3w4:variants/ch3w4/libdfm.so}; do
    n=${v%%:*}; l=${v#*:}
    c2 ${n}_$r $l || exit 1
    DFM_NO_LANES=1 c2 ${n}_solo_$r $l || exit 1
  done
done
for v in ${CHOW_TEST:-ch3:variants/ch3/libdfm.so ch3w4:variants/ch3w4/libdfm.so}; do
  n=${v%%:*}; export DFM_LIB_PATH=${v#*:}
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_production.py -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest_$n.txt 2>&1
  rc=$?; echo "pytest $n rc=$rc"; tail -2 $OUT/pytest_$n.txt; [ $rc -eq 0 ] || exit 1
done
