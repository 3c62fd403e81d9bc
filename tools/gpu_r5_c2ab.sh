# round 5: C2 direct-solver strong-filter schedule A/B (DFM_DIRECT_D0 / DFM_DIRECT_CYC), then the GPU suite
OUT=gpurun_out/c2ab
mkdir -p $OUT
c2() { env "$@" timeout -k 10 200 python3 -u tools/bench_configs.py --configs c2 --reps 5 > $OUT/c2.jsonl 2> $OUT/c2.err || { echo "c2 rc=$?"; tail -5 $OUT/c2.err; return 1; }
python3 -c "import json; d=json.loads(open('$OUT/c2.jsonl').readline()); print('$*', d['value'], d['ms_per_job'], d['eig_iterations'], d['kernels_ms_per_job'])"; }
c2 DFM_DIRECT_D0=4 DFM_DIRECT_CYC=4 && c2 DFM_DIRECT_D0=5 DFM_DIRECT_CYC=3 && c2 DFM_DIRECT_D0=4 DFM_DIRECT_CYC=4 && c2 DFM_DIRECT_D0=5 DFM_DIRECT_CYC=3 || exit 1
# Chow timing diagnostics (one lane, solo kernels): production vs tile 0 staged once (no staging rhythm) vs no gathered loads
c2 DFM_NO_LANES=1 && c2 DFM_NO_LANES=1 DFM_LIB_PATH=variants/ch_ns/libdfm.so && c2 DFM_NO_LANES=1 DFM_LIB_PATH=variants/ch_nl/libdfm.so || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $OUT/pytest.txt 2>&1; echo pytest_rc=$?; tail -3 $OUT/pytest.txt
