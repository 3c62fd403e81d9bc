"""Per-launch durations (in order) of the C3 hot loop from a rocprofv3 kernel trace."""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: n.split("(")[0].replace("void ", "").replace("dfm::", "")[:40]
seq = [(short(r["Kernel_Name"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
        int(r["Start_Timestamp"])) for r in rows]
# last step only: from the last boot_prep to the end
last = max(i for i, s in enumerate(seq) if s[0].startswith("boot_prep"))
t0 = seq[last][2]
tot = collections.Counter()
for name, us, st in seq[last:]:
    print(f"{(st - t0) / 1e3:9.1f} us  {us:9.1f} us  {name}")
    tot[name] += us
print("---")
for k, v in tot.most_common(): print(f"{v:10.1f} us  {k}")
