# round 5: the whole -m gpu suite, then the default bench line (one call)
mkdir -p gpurun_out/full
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/full/pytest.txt 2>&1
rc=$?; echo pytest_rc=$rc; tail -4 gpurun_out/full/pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/full/bench.json 2> gpurun_out/full/bench.err; echo bench_rc=$?
python - <<'P'
import json; r=json.load(open("gpurun_out/full/bench.json"))
print(r["value"], r["ms_per_step"], r["roofline"]["frac"], r.get("all_fields",{}).get("value"), r["cpu_baseline"]["value"])
P
