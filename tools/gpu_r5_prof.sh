# round 5: GPU suite, then a rocprofv3 kernel-trace summary of the default bench (headline launches only)
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/prof/pytest.txt 2>&1
rc=$?; echo pytest_rc=$rc; tail -3 gpurun_out/prof/pytest.txt
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/rp -o run -- python3 bench.py --no-cpu-baseline --no-all-fields --steps 10 > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err; echo prof_rc=$?
find gpurun_out/prof/rp -name "*kernel_stats.csv" | head -3
