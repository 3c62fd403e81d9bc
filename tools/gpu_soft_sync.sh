#!/bin/bash
# Lasso host-side stall probe: back-to-back soft selections under three
# settings (spin timeout 700 ms; 2 s; 2 s with a polling host wait), each
# reporting lasso_stats and every slow launch (host time vs kernel time).
OUT=${1:-gpurun_out/softsync}
N=${2:-150}
mkdir -p "$OUT"
export TMPDIR=/tmp
DFM_LASSO_TMO_MS=700 timeout -k 10 300 python3 -u tools/soft_repeat.py "$N" > "$OUT/tmo700.out" 2> "$OUT/tmo700.err" || exit 1
tail -3 "$OUT/tmo700.out"; grep -m3 "host" "$OUT/tmo700.err"
DFM_LASSO_TMO_MS=2000 DFM_LASSO_SYNC_POLL=1 timeout -k 10 300 python3 -u tools/soft_repeat.py "$N" > "$OUT/poll.out" 2> "$OUT/poll.err" || exit 1
tail -3 "$OUT/poll.out"; grep -m3 "host" "$OUT/poll.err"
DFM_LASSO_TMO_MS=2000 timeout -k 10 300 python3 -u tools/soft_repeat.py "$N" > "$OUT/tmo2000.out" 2> "$OUT/tmo2000.err" || exit 1
tail -3 "$OUT/tmo2000.out"; grep -m3 "host" "$OUT/tmo2000.err"
