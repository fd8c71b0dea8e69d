#!/bin/bash
# Display groups in flight (THESIA_RENDER_STREAMS 2 / 3 / 4) on the C5 line, two interleaved rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05_rstreams}
mkdir -p $O
for r in 1 2; do
  for n in 2 3 4; do
    THESIA_RENDER_STREAMS=$n timeout -k 10 200 python bench.py --workload c5 --no-exact > $O/s${n}_$r.json 2> $O/s${n}_$r.err || exit 1
  done
done
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for r in (1, 2):
    for n in (2, 3, 4):
        d = json.loads(open(f"{o}/s{n}_{r}.json").read().strip().splitlines()[-1])
        print("streams", n, "round", r, "step %.3f" % d["ms_per_step"], "display %.3f" % d["roofline_display"]["display_ms"])
PY
