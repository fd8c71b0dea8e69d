#!/bin/bash
# Round 4: the display groups' stream scheduling: the stripe groups' cost factor (1, 3, 5) on the
# experiment build, C5 line with 4 render streams, interleaved, two rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_aa}
mkdir -p $O
export THESIA_LIB=$R/multi-spectrogram-viewer_amd/lib/libthesia_exp.so
for r in 1 2; do
  for f in 1 3 5; do
    THESIA_STRIPE_COST=$f timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 2 --render-paths 0 > $O/c5_${f}_$r.json 2> $O/c5_${f}_$r.err || { tail -5 $O/c5_${f}_$r.err; exit 1; }
    tail -1 $O/c5_${f}_$r.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('factor $f round $r', round(d['ms_per_step'],3), round(d['roofline_display']['display_ms'],3))"
    grep render_paths $O/c5_${f}_$r.json | cut -c1-120
  done
done
echo done
