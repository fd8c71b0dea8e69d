#!/bin/bash
# amp dB kind at compile time in stft5 (canonical + viewer geometry) and stft3v (viewer
# geometries, no range fold) vs the run-time kind (THESIA_STFT3_RTKIND, experiment library).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05_kd2}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_viewer_geometry.py tests/test_gpu_multitrack.py tests/test_gpu_configs.py tests/test_gpu_stft.py > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
X="--no-cpu-baseline --no-exact --no-e2e --no-rfft-roofline --no-c1"
E=multi-spectrogram-viewer_amd/lib/libthesia_exp.so
for r in 1 2; do
  for v in ct rt; do
    if [ $v = rt ]; then export THESIA_STFT3_RTKIND=1; else unset THESIA_STFT3_RTKIND; fi
    THESIA_LIB=$E timeout -k 10 200 python bench.py --workload viewer $X > $O/viewer_${v}_$r.json 2> $O/viewer_${v}_$r.err || exit 1
    THESIA_LIB=$E timeout -k 10 200 python bench.py --output amp_db $X > $O/c4amp_${v}_$r.json 2> $O/c4amp_${v}_$r.err || exit 1
    THESIA_LIB=$E timeout -k 10 200 python bench.py --output amp_db --win 1920 --hop 480 --kernels 3,5 $X > $O/view48_${v}_$r.json 2> $O/view48_${v}_$r.err || exit 1
  done
done
unset THESIA_STFT3_RTKIND
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for w in ("viewer", "c4amp", "view48"):
    for r in (1, 2):
        for v in ("ct", "rt"):
            ls = [json.loads(x) for x in open(f"{o}/{w}_{v}_{r}.json").read().strip().splitlines() if x.startswith("{")]
            d = ls[-1]
            extra = {k: x[k] for x in ls for k in x if k == "kernels_ms"}
            print(w, v, r, "ms/step %.4f" % d["ms_per_step"], json.dumps(extra)[:300])
PY
