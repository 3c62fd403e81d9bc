"""HBM traffic per kernel launch from two rocprofv3 PMC passes.

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR > profiles/rNN_pmc_traffic.json

FETCH_DIR holds the `--pmc FETCH_SIZE -f csv` pass, WRITE_DIR the
`--pmc WRITE_SIZE -f csv` pass (separate passes: FETCH_SIZE takes 3 of the 4
TCC slots, WRITE_SIZE 2).  Both counters are in KiB (counter_defs.yaml).  On
gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced read
(MI355X_MICROARCH.md, HBM section), so HBM bytes per launch =
2 * 1024 * FETCH_SIZE + 1024 * WRITE_SIZE, averaged over the launches of each
kernel.  Infinity-Cache hits are counted as fetches by these counters."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def read_pass(d, counter):
    per = defaultdict(dict)   # kernel -> dispatch id -> value
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "?")
                did = row.get("Dispatch_Id") or row.get("Correlation_Id") or str(len(per[name]))
                per[name][did] = per[name].get(did, 0.0) + float(row["Counter_Value"])
    return per


def short(name):
    base = name.split("(")[0]
    return base.replace("void ", "").replace("dfm::", "").strip()


def main():
    fetch = read_pass(sys.argv[1], "FETCH_SIZE")
    write = read_pass(sys.argv[2], "WRITE_SIZE")
    out = {}
    for name in sorted(set(fetch) | set(write)):
        f = list(fetch.get(name, {}).values())
        w = list(write.get(name, {}).values())
        fa = sum(f) / len(f) if f else None
        wa = sum(w) / len(w) if w else None
        rec = {"launches_fetch_pass": len(f), "launches_write_pass": len(w),
               "fetch_size_kib_avg": fa, "write_size_kib_avg": wa}
        if fa is not None and wa is not None:
            rec["hbm_bytes_per_launch"] = 2 * 1024 * fa + 1024 * wa
        out[short(name)] = rec
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
