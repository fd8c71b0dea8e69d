#!/bin/bash
# The run-time-kind instances with one kind switch per frame (compile-time kind bodies) against
# the previous per-bin branches is not A/B-able in one library; this records the parity suites
# and the power-dB / magnitude lines (C2's kind) after the change, to set beside r05_kd2's.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r05_kd3}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_streaming.py tests/test_gpu_ranges.py tests/test_gpu_stft.py tests/test_gpu_configs.py tests/test_gpu_viewer_geometry.py > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
X="--no-cpu-baseline --no-exact --no-e2e --no-rfft-roofline --no-c1"
for o in power_db amp_db; do
  timeout -k 10 200 python bench.py --output $o --kernels 3,5 $X > $O/c4_$o.json 2> $O/c4_$o.err || exit 1
done
# the run-time-kind instances on amp dB (r05_kd2's rt: 5.62 ms stft5 with per-bin branches)
THESIA_STFT3_RTKIND=1 THESIA_LIB=multi-spectrogram-viewer_amd/lib/libthesia_exp.so timeout -k 10 200 \
  python bench.py --output amp_db --kernels 3,5 $X > $O/c4_rt_amp_db.json 2> $O/c4_rt_amp_db.err || exit 1
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for w in ("power_db", "amp_db", "rt_amp_db"):
    ls = [json.loads(x) for x in open(f"{o}/c4_{w}.json").read().strip().splitlines() if x.startswith("{")]
    k = [x["kernels_ms"] for x in ls if "kernels_ms" in x]
    print(w, "ms/step %.4f" % ls[-1]["ms_per_step"], k[0] if k else "")
PY
