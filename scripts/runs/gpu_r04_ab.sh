#!/bin/bash
# Round 4: stripe kernel timing ablations (experiment build, THESIA_STRIPE_ABL: 1 no staging past
# the first chunk, 2 no emission, 4 no horizontal sums), per group alone at the C5 geometry.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_ab}
mkdir -p $O
cd /tmp
export THESIA_LIB=$R/multi-spectrogram-viewer_amd/lib/libthesia_exp.so THESIA_RENDER_STREAMS=1
for a in 0 1 2 4 7; do
  THESIA_STRIPE_ABL=$a timeout -k 10 300 python3 $R/scripts/display_groups_ab.py 0 > $O/groups_abl$a.txt 2>&1 || { tail $O/groups_abl$a.txt; exit 1; }
  echo "abl $a: $(tail -1 $O/groups_abl$a.txt | python3 -c "import json,sys; d=json.load(sys.stdin)['display_us_per_group']; print({k: v['0'] for k, v in d.items() if k in ('44100/256','48000/512','22050/256')})")"
done
echo done
