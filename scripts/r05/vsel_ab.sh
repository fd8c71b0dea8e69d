#!/bin/bash
# The full GPU suite on the product library, then grey_vert's x4 staging with selected-address
# stores (product) vs exec-masked stores (THESIA_VSTAGE_MASKED, experiment library) on the C5 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05_vsel}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -20 $O/gpu_tests.txt; exit 1; }
tail -2 $O/gpu_tests.txt
E=multi-spectrogram-viewer_amd/lib/libthesia_exp.so
for r in 1 2 3; do
  unset THESIA_VSTAGE_MASKED
  THESIA_LIB=$E timeout -k 10 200 python bench.py --workload c5 --no-exact > $O/sel_$r.json 2> $O/sel_$r.err || exit 1
  export THESIA_VSTAGE_MASKED=1
  THESIA_LIB=$E timeout -k 10 200 python bench.py --workload c5 --no-exact > $O/msk_$r.json 2> $O/msk_$r.err || exit 1
done
unset THESIA_VSTAGE_MASKED
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for r in (1, 2, 3):
    for v in ("sel", "msk"):
        d = json.loads(open(f"{o}/{v}_{r}.json").read().strip().splitlines()[-1])
        print(v, r, "step %.3f" % d["ms_per_step"], "display %.3f" % d["roofline_display"]["display_ms"],
              "spectrogram %.3f" % d["roofline"]["overlapped_ms"])
PY
