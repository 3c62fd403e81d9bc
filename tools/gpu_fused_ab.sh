#!/bin/bash
# Fused direct eigensolver session: the -m gpu suite with the fused path (the
# default), then the C2 config line with DFM_EIG_FUSED=1 / 0 and a rocprofv3
# kernel summary of the fused C2 job.  Each step bounded; stop on failure.
OUT=${1:-gpurun_out/fz}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
tail -15 "$OUT/pytest.log"
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
for F in 1 0; do
  DFM_EIG_FUSED=$F timeout -k 10 300 python3 -u tools/bench_configs.py --configs c2 --reps 5 > "$OUT/c2_f$F.jsonl" 2> "$OUT/c2_f$F.err" || { echo "c2 f$F rc=$?"; tail -5 "$OUT/c2_f$F.err"; exit 1; }
  cut -c1-400 "$OUT/c2_f$F.jsonl"
done
DFM_EIG_PROF=1 timeout -k 10 300 python3 -u tools/bench_configs.py --configs c2 --reps 2 > "$OUT/c2_prof.jsonl" 2> "$OUT/c2_prof.err" || { echo "c2 prof rc=$?"; tail -5 "$OUT/c2_prof.err"; exit 1; }
grep eig_fused "$OUT/c2_prof.err" | tail -6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/c2trace" -o run -- python3 tools/bench_configs.py --configs c2 --reps 3 > "$OUT/c2trace.out" 2> "$OUT/c2trace.err" || { echo "c2 trace rc=$?"; tail -5 "$OUT/c2trace.err"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/c2trace/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:16]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['TotalDurationNs'])/1e6:8.2f} ms {float(r['AverageNs'])/1e3:8.1f} us")
PY
