# round 5: is the H.Z GEMM bound by its LDS-DMA staging?  per-launch durations of gemmh_kernel_t (rocprofv3 kernel
# trace): production vs variants/gA (B tiles staged only for the first stages: A traffic only) and variants/gB
# (A tiles staged only for the first stages); both variants compute WRONG values (timing only)
OUT=gpurun_out/gemmdiag
mkdir -p $OUT
export TMPDIR=/tmp
for v in prod gA gB; do
  if [ $v = prod ]; then unset DFM_LIB_PATH; else export DFM_LIB_PATH=variants/$v/libdfm.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT/$v -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-all-fields > $OUT/$v.json 2> $OUT/$v.err; echo $v=$?
  python3 - $OUT/$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
v = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f)) if "gemmh" in r["Kernel_Name"])
print(sys.argv[1].split("/")[-1], "gemmh launches", len(v), "top8 us", [round(x, 1) for x in v[-8:]])
PY
done
unset DFM_LIB_PATH
