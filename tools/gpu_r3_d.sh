#!/bin/bash
# Round-3 session D: C2 timing with the row-split Chow kernel, the C2
# tolerance/accuracy probe, shard-size sweep (strong-scaling projection), SQ
# stall counters of the C3 passes.  Exit other than 0/1 stops.
OUT=${1:-gpurun_out/d}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then tail -30 "$OUT/$name.err"; exit $rc; fi
  return 0
}
step c2 200 python -u tools/bench_configs.py --configs c2 --reps 3
cat "$OUT/c2.out"
step c2tol 300 python -u tools/c2_tol_probe.py
cat "$OUT/c2tol.out"
for R in 1250 2500 5000; do
  step shard_$R 120 python -u bench.py --no-cpu-baseline --replicates $R --steps 10 --warmup 3
  python3 -c "import json; d=json.loads(open('$OUT/shard_$R.out').read().strip().splitlines()[-1]); print('shard', $R, d['ms_per_step'], d['kernels_ms'])"
done
step sq 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM --kernel-include-regex "boot_|gemmh|eig_small" -f csv -d "$OUT/sq" -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
step grbm 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-include-regex "gemmh|boot_ap2" -f csv -d "$OUT/grbm" -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline
echo ALLDONE
