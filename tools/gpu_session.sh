#!/bin/bash
# One parameterised GPU measurement session (replaces round 5's one-off
# tools/gpu_r5_*.sh scripts).  Run on the box through gpurun, e.g.
#   gpurun -- 'bash tools/gpu_session.sh r06a tests bench prof pmc shards configs'
# Usage: tools/gpu_session.sh TAG STEP...   (output under gpurun_out/TAG)
# Steps (each under its own time limit; the session stops at the first failure):
#   tests      the -m gpu suite (pytest.txt)
#   bench      the default bench line (bench.json)
#   prof       rocprofv3 --kernel-trace --stats of the headline workload (prof/)
#   trace      per-dispatch kernel trace of a 3-step C3 run (TRACE_ARGS: extra bench.py flags)
#   pmc        FETCH_SIZE and WRITE_SIZE passes of the C3 GEMM + passes -> pmc_traffic.json
#   pmc_c2     FETCH_SIZE / WRITE_SIZE of the C2 job's fused solver + Chow, one lane
#              (DFM_NO_LANES=1: per-launch bytes cover more replicates than a lane launch) -> pmc_traffic_c2.json
#   sq_c2      SQ counter passes of the C2 kernels (one lane: DFM_NO_LANES=1)
#   sq_c3      SQ / TA / TCP counter passes of the C3 per-replicate passes (KRE: kernel regex)
#   ta_c2      TA / TCP counters of every C2 kernel (one lane)
#   shards     C3 at 1250 / 2500 / 5000 / 9999 replicates (shards.jsonl)
#   configs    tools/bench_configs.py c1,c2,c4,c5 (configs.jsonl)
#   c2         C2 only, 5 reps (c2.jsonl)
#   c2prof     rocprofv3 kernel summary of the C2 job, one lane (c2prof/)
#   c5         bench.py --workload c5, expanding and rolling 1000 (c5.jsonl)
#   abrows     production vs $VAR: C3 rows bit-identical + alternating timings (3 rounds)
#   ab         production vs $VAR (a variant libdfm.so) alternating, C3 + 1250 (+ C2 if C2=1)
#   sanitize   the host sanitizer harnesses (tools/gpu_sanitize.sh)
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
fail() { echo "$1 rc=$2"; [ -f "$3" ] && tail -5 "$3"; exit 1; }
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d.get('value'), d.get('ms_per_step', d.get('ms_per_job')), (d.get('roofline') or {}).get('frac'))" "$@" || true; }
bench_ab() {   # name lib args...
  local name=$1 lib=$2; shift 2
  if [ "$lib" = "-" ]; then unset DFM_LIB_PATH; else export DFM_LIB_PATH=$lib; fi
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --no-all-fields "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" \
    || fail "$name" $? "$OUT/$name.err"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['kernels_ms'], [(h['kernel'][:14], h['frac']) for h in d.get('roofline_hbm', [])], d['roofline']['frac'])" "$OUT/$name.json" "$name"
  unset DFM_LIB_PATH
}
c2_ab() {
  local name=$1 lib=$2
  if [ "$lib" = "-" ]; then unset DFM_LIB_PATH; else export DFM_LIB_PATH=$lib; fi
  timeout -k 10 200 python3 -u tools/bench_configs.py --configs c2 --reps 5 > "$OUT/$name.jsonl" 2> "$OUT/$name.err" \
    || fail "$name" $? "$OUT/$name.err"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).readline()); print(sys.argv[2], d['value'], d['ms_per_job'], d.get('kernels_ms_per_job'))" "$OUT/$name.jsonl" "$name"
  unset DFM_LIB_PATH
}
for step in "$@"; do
  echo "== $step"
  case $step in
    tests)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.txt" 2>&1 \
        || fail tests $? "$OUT/pytest.txt"
      tail -2 "$OUT/pytest.txt" ;;
    bench)
      timeout -k 10 300 python3 -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || fail bench $? "$OUT/bench.err"
      line "$OUT/bench.json" bench ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- python3 bench.py \
        --no-cpu-baseline --no-all-fields > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" || fail prof $? "$OUT/bench_prof.err"
      line "$OUT/bench_prof.json" bench_under_rocprof ;;
    trace)   # per-dispatch kernel trace of a short C3 run (trace/: kernel_trace.csv)
      timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d "$OUT/trace" -o run -- python3 bench.py --steps 3 --warmup 2 \
        --no-cpu-baseline --no-all-fields ${TRACE_ARGS} > "$OUT/trace.json" 2> "$OUT/trace.err" || fail trace $? "$OUT/trace.err"
      line "$OUT/trace.json" bench_under_trace ;;
    pmc)
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "gemmh_|boot_" -f csv -d "$OUT/pmc_f" \
        -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-all-fields > "$OUT/pmc_f.out" 2> "$OUT/pmc_f.err" \
        || fail pmc_f $? "$OUT/pmc_f.err"
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "gemmh_|boot_" -f csv -d "$OUT/pmc_w" \
        -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-all-fields > "$OUT/pmc_w.out" 2> "$OUT/pmc_w.err" \
        || fail pmc_w $? "$OUT/pmc_w.err"
      python3 tools/pmc_traffic.py "$OUT/pmc_f" "$OUT/pmc_w" > "$OUT/pmc_traffic.json" && head -c 1200 "$OUT/pmc_traffic.json"; echo ;;
    pmc_c2)
      export DFM_NO_LANES=1
      timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "eig_fused|chow_all" -f csv -d "$OUT/pmc2_f" \
        -o run -- python3 tools/bench_configs.py --configs c2 --reps 1 > "$OUT/pmc2_f.out" 2> "$OUT/pmc2_f.err" \
        || fail pmc2_f $? "$OUT/pmc2_f.err"
      timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "eig_fused|chow_all" -f csv -d "$OUT/pmc2_w" \
        -o run -- python3 tools/bench_configs.py --configs c2 --reps 1 > "$OUT/pmc2_w.out" 2> "$OUT/pmc2_w.err" \
        || fail pmc2_w $? "$OUT/pmc2_w.err"
      unset DFM_NO_LANES
      python3 tools/pmc_traffic.py "$OUT/pmc2_f" "$OUT/pmc2_w" > "$OUT/pmc_traffic_c2.json" && head -c 1200 "$OUT/pmc_traffic_c2.json"; echo ;;
    sq_c3)   # SQ / TA / TCP counter passes of the C3 passes (KRE: kernel regex, default the per-replicate passes)
      KRE=${KRE:-boot_}
      timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "$KRE" -f csv -d "$OUT/sq3a" -o run -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-all-fields > "$OUT/sq3a.out" 2> "$OUT/sq3a.err" \
        || fail sq3a $? "$OUT/sq3a.err"
      timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ \
        GRBM_GUI_ACTIVE --kernel-include-regex "$KRE" -f csv -d "$OUT/sq3b" -o run -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-all-fields > "$OUT/sq3b.out" 2> "$OUT/sq3b.err" \
        || fail sq3b $? "$OUT/sq3b.err" ;;
    ta_c2)   # TA / TCP counters of every C2 kernel (one lane)
      export DFM_NO_LANES=1
      timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY TA_FLAT_READ_WAVEFRONTS TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ \
        GRBM_GUI_ACTIVE -f csv -d "$OUT/ta2" -o run -- python3 tools/bench_configs.py --configs c2 --reps 1 \
        > "$OUT/ta2.out" 2> "$OUT/ta2.err" || fail ta2 $? "$OUT/ta2.err"
      unset DFM_NO_LANES ;;
    sq_c2)
      export DFM_NO_LANES=1
      timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
        SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM --kernel-include-regex "chow_all|eig_fused" -f csv \
        -d "$OUT/sq1" -o run -- python3 tools/bench_configs.py --configs c2 --reps 1 > "$OUT/sq1.out" 2> "$OUT/sq1.err" \
        || fail sq1 $? "$OUT/sq1.err"
      timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
        SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU --kernel-include-regex "chow_all|eig_fused" -f csv -d "$OUT/sq2" -o run -- \
        python3 tools/bench_configs.py --configs c2 --reps 1 > "$OUT/sq2.out" 2> "$OUT/sq2.err" || fail sq2 $? "$OUT/sq2.err"
      unset DFM_NO_LANES ;;
    shards)
      : > "$OUT/shards.jsonl"
      for n in 1250 2500 5000 9999; do
        timeout -k 10 200 python3 -u bench.py --replicates $n --no-cpu-baseline --no-all-fields > "$OUT/s$n.json" \
          2> "$OUT/s$n.err" || fail "s$n" $? "$OUT/s$n.err"
        tail -1 "$OUT/s$n.json" >> "$OUT/shards.jsonl"; line "$OUT/s$n.json" "shard$n"
      done ;;
    configs)
      timeout -k 10 400 python3 -u tools/bench_configs.py --configs c1,c2,c4,c5 --reps 5 > "$OUT/configs.jsonl" \
        2> "$OUT/configs.err" || fail configs $? "$OUT/configs.err"
      cut -c1-300 "$OUT/configs.jsonl" ;;
    c2)
      c2_ab c2 - ;;
    c2prof)
      export DFM_NO_LANES=1
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/c2prof" -o run -- python3 tools/bench_configs.py \
        --configs c2 --reps 5 > "$OUT/c2prof.jsonl" 2> "$OUT/c2prof.err" || fail c2prof $? "$OUT/c2prof.err"
      unset DFM_NO_LANES ;;
    c5)
      timeout -k 10 300 python3 -u bench.py --workload c5 > "$OUT/c5.jsonl" 2> "$OUT/c5.err" || fail c5 $? "$OUT/c5.err"
      timeout -k 10 300 python3 -u bench.py --workload c5 --rolling 1000 >> "$OUT/c5.jsonl" 2>> "$OUT/c5.err" \
        || fail c5r $? "$OUT/c5.err"
      cut -c1-300 "$OUT/c5.jsonl" ;;
    ab)
      for r in 1 2; do
        bench_ab "new_$r" - && bench_ab "var_$r" "$VAR"
        bench_ab "new1250_$r" - --replicates 1250 && bench_ab "var1250_$r" "$VAR" --replicates 1250
        if [ "$C2" = 1 ]; then c2_ab "newc2_$r" - && c2_ab "varc2_$r" "$VAR"; fi
      done ;;
    abrows)   # production vs $VAR: C3 rows bit-identical, then alternating timings (C3 + 1250)
      bench_ab var_rows "$VAR" --steps 2 --warmup 1 --dump-rows "$OUT/rows_var.npy"
      bench_ab new_rows - --steps 2 --warmup 1 --dump-rows "$OUT/rows_new.npy"
      python3 -c "import numpy as np,sys; a=np.load(sys.argv[1]); b=np.load(sys.argv[2]); print('rows bit-identical:', a.shape, np.array_equal(a, b), float(np.nanmax(np.abs(a-b))))" "$OUT/rows_var.npy" "$OUT/rows_new.npy"
      for r in 1 2 3; do
        bench_ab "var_$r" "$VAR" && bench_ab "new_$r" -
        bench_ab "var1250_$r" "$VAR" --replicates 1250 && bench_ab "new1250_$r" - --replicates 1250
      done ;;
    sanitize)
      bash tools/gpu_sanitize.sh ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== session $TAG done"
