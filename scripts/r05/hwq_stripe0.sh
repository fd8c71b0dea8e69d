#!/bin/bash
# The display's queue regime (experiment library, C5 line, two rounds): default (4 hardware
# queues: the 4 library streams share 2), GPU_MAX_HW_QUEUES=8 (4 distinct queues), and 8 queues
# with the stripe groups serialised on one stream (THESIA_RENDER_STRIPE0: a temporary hook in
# engine.cpp, removed after the measurement; profiles/r05_hwq2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05_hwq2}
mkdir -p $O
E=multi-spectrogram-viewer_amd/lib/libthesia_exp.so
for r in 1 2; do
  THESIA_LIB=$E timeout -k 10 200 python bench.py --workload c5 --no-exact > $O/q4_$r.json 2> $O/q4_$r.err || exit 1
  GPU_MAX_HW_QUEUES=8 THESIA_LIB=$E timeout -k 10 200 python bench.py --workload c5 --no-exact > $O/q8_$r.json 2> $O/q8_$r.err || exit 1
  THESIA_RENDER_STRIPE0=1 GPU_MAX_HW_QUEUES=8 THESIA_LIB=$E timeout -k 10 200 python bench.py --workload c5 --no-exact > $O/q8s_$r.json 2> $O/q8s_$r.err || exit 1
  THESIA_RENDER_STRIPE0=1 THESIA_LIB=$E timeout -k 10 200 python bench.py --workload c5 --no-exact > $O/q4s_$r.json 2> $O/q4s_$r.err || exit 1
done
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for r in (1, 2):
    for v in ("q4", "q8", "q8s", "q4s"):
        d = json.loads(open(f"{o}/{v}_{r}.json").read().strip().splitlines()[-1])
        print(v, r, "step %.3f" % d["ms_per_step"], "display %.3f" % d["roofline_display"]["display_ms"],
              "spectrogram %.3f" % d["roofline"]["overlapped_ms"])
PY
