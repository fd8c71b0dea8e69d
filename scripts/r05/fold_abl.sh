#!/bin/bash
# Ablation: the C5 spectrogram batches with and without the compiled-in range fold
# (THESIA_STFT3_NOFOLD, experiment library: ranges not written, timing only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05_fold}
mkdir -p $O
E=multi-spectrogram-viewer_amd/lib/libthesia_exp.so
for r in 1 2; do
  unset THESIA_STFT3_NOFOLD
  THESIA_LIB=$E timeout -k 10 200 python bench.py --workload c5 --no-exact > $O/fold_$r.json 2> $O/fold_$r.err || exit 1
  export THESIA_STFT3_NOFOLD=1
  THESIA_LIB=$E timeout -k 10 200 python bench.py --workload c5 --no-exact > $O/nofold_$r.json 2> $O/nofold_$r.err || exit 1
done
unset THESIA_STFT3_NOFOLD
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for r in (1, 2):
    for v in ("fold", "nofold"):
        d = json.loads(open(f"{o}/{v}_{r}.json").read().strip().splitlines()[-1])
        rf = d["roofline"]
        print(v, r, "spectrogram %.3f" % rf["overlapped_ms"], [round(b["kernel_ms"], 3) for b in rf["per_batch"]])
PY
