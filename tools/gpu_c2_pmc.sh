#!/bin/bash
# SQ counters of the C2 job's Chow and fused eigen kernels (one --pmc pass,
# kernel-trace only): instruction mix and wait cycles per kernel.
OUT=${1:-gpurun_out/c2pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --kernel-include-regex "chow_all|eig_fused" -f csv -d "$OUT/pmc" -o run -- python3 tools/bench_configs.py --configs c2 --reps 1 > "$OUT/pmc.out" 2> "$OUT/pmc.err"
rc=$?
echo "pmc rc=$rc"; tail -3 "$OUT/pmc.err"
python3 - "$OUT" <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for f in glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[k].add(r.get("Dispatch_Id"))
for k, d in acc.items():
    print(k, len(n[k]), {c: round(v / max(1, len(n[k])), 1) for c, v in sorted(d.items())})
PY
