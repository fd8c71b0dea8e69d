#!/bin/bash
# stft3 amp dB with the kind / range fold at compile time vs at run time (THESIA_STFT3_RTKIND,
# experiment library): parity tests on the product library, then the C5 line interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05_kd}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_streaming.py tests/test_gpu_ranges.py tests/test_gpu_parity.py > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for r in 1 2 3; do
  THESIA_LIB=multi-spectrogram-viewer_amd/lib/libthesia_exp.so timeout -k 10 200 python bench.py --workload c5 --no-exact > $O/ct_$r.json 2> $O/ct_$r.err || exit 1
  THESIA_STFT3_RTKIND=1 THESIA_LIB=multi-spectrogram-viewer_amd/lib/libthesia_exp.so timeout -k 10 200 python bench.py --workload c5 --no-exact > $O/rt_$r.json 2> $O/rt_$r.err || exit 1
done
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for r in (1, 2, 3):
    for v in ("ct", "rt"):
        d = json.loads(open(f"{o}/{v}_{r}.json").read().strip().splitlines()[-1])
        rf = d["roofline"]
        print(v, r, "step %.3f" % d["ms_per_step"], "spec %.3f" % rf["overlapped_ms"],
              [round(b["kernel_ms"], 3) for b in rf["per_batch"]])
PY
