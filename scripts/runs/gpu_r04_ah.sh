#!/bin/bash
# Round 4: C5 line with the device-side range (default) vs the host exchange (THESIA_HOST_RANGE=1),
# separate processes, three interleaved rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_ah}
mkdir -p $O
for r in 1 2 3; do
  for h in 0 1; do
    THESIA_HOST_RANGE=$h timeout -k 10 300 python3 bench.py --workload c5 --steps 20 --warmup 3 > $O/c5_h${h}_$r.json 2> $O/c5_h${h}_$r.err || { tail -5 $O/c5_h${h}_$r.err; exit 1; }
    tail -1 $O/c5_h${h}_$r.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('host_range $h round $r', round(d['ms_per_step'],3), round(d['roofline_display']['display_ms'],3))"
  done
done
echo done
