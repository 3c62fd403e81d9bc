# round 5: is ap2 bound by its Q / Y tile loads?  per-launch durations of boot_ap2_kernel (rocprofv3 kernel trace),
# production vs variants/ap2nl (DFM_AP2_DIAG_NOLOAD: no tile loads, wrong results, timing only)
OUT=gpurun_out/ap2diag
mkdir -p $OUT
export TMPDIR=/tmp
for v in prod nl; do
  if [ $v = nl ]; then export DFM_LIB_PATH=variants/ap2nl/libdfm.so; else unset DFM_LIB_PATH; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -f csv -d $OUT/$v -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-all-fields > $OUT/$v.json 2> $OUT/$v.err; echo $v=$?
  python3 - $OUT/$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = {}
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    for k in ("boot_ap2", "boot_y2", "boot_cheb_mid", "boot_cheb_kernel", "gemmh"):
        if k in n:
            d.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    print(sys.argv[1].split("/")[-1], k, len(v), "max %.1f us" % max(v), "top5", sorted(v)[-5:])
PY
done
unset DFM_LIB_PATH
