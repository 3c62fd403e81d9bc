#!/bin/bash
# Lasso host-side stall probe: back-to-back soft selections under four
# settings (spin timeout 700 ms; 2 s with a polling host wait; 2 s with
# ROCr's scratch reclaim off; 2 s), each reporting lasso_stats and every slow
# launch (host time vs kernel time).
OUT=${1:-gpurun_out/softsync}
N=${2:-150}
mkdir -p "$OUT"
export TMPDIR=/tmp
DFM_LASSO_TMO_MS=700 timeout -k 10 300 python3 -u tools/soft_repeat.py "$N" > "$OUT/tmo700.out" 2> "$OUT/tmo700.err" || exit 1
tail -3 "$OUT/tmo700.out"; grep -m3 "host" "$OUT/tmo700.err"
DFM_LASSO_TMO_MS=2000 DFM_LASSO_SYNC_POLL=1 timeout -k 10 300 python3 -u tools/soft_repeat.py "$N" > "$OUT/poll.out" 2> "$OUT/poll.err" || exit 1
tail -3 "$OUT/poll.out"; grep -m3 "host" "$OUT/poll.err"
HSA_NO_SCRATCH_RECLAIM=1 DFM_LASSO_TMO_MS=2000 timeout -k 10 300 python3 -u tools/soft_repeat.py "$N" > "$OUT/noreclaim.out" 2> "$OUT/noreclaim.err" || exit 1
tail -3 "$OUT/noreclaim.out"; grep -m3 "host" "$OUT/noreclaim.err"
DFM_LASSO_TMO_MS=2000 timeout -k 10 300 python3 -u tools/soft_repeat.py "$N" > "$OUT/tmo2000.out" 2> "$OUT/tmo2000.err" || exit 1
tail -3 "$OUT/tmo2000.out"; grep -m3 "host" "$OUT/tmo2000.err"
