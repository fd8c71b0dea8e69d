#!/bin/bash
# C5 steps for each library variant in multi-spectrogram-viewer_amd/lib/vd/*.so (THESIA_LIB), the
# render byte tests on each first, then ROUNDS alternating rounds of STEPS steps (separate
# processes). BENCH_ARGS: extra bench.py arguments.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${1:-lib_ab}; mkdir -p $O
for lib in $R/multi-spectrogram-viewer_amd/lib/vd/*.so; do
  n=$(basename $lib .so)
  THESIA_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -q -x -k "render or ragged or image" --timeout 240 --timeout-method thread > $O/pytest_$n.txt 2>&1 || { tail -20 $O/pytest_$n.txt; exit 1; }
  echo "$n: $(tail -1 $O/pytest_$n.txt)"
done
for r in $(seq ${ROUNDS:-3}); do
for lib in $R/multi-spectrogram-viewer_amd/lib/vd/*.so; do
  n=$(basename $lib .so)
  THESIA_LIB=$lib timeout -k 10 200 python3 bench.py --workload c5 --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > $O/b_${n}_$r.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$O/b_${n}_$r.log').read().strip().splitlines()[-1]); print('$r', '$n', 'display', round(d['roofline_display']['display_ms'], 3), 'spec', round(d['roofline']['overlapped_ms'], 3), 'step', round(d['ms_per_step'], 3))"
done
done
