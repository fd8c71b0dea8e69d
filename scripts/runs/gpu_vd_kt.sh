#!/bin/bash
# Per-group display kernel times (rocprofv3 kernel trace) for each display variant library
# (scripts/build_variant_display.sh), one C5 bench process each; the ragged-group byte tests on
# every variant first. BENCH_ARGS: extra bench.py arguments (e.g. --render-path 3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${1:-vd_kt}; mkdir -p $O
export TMPDIR=/tmp
for lib in $R/multi-spectrogram-viewer_amd/lib/vd/*.so; do
  n=$(basename $lib .so)
  THESIA_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -q -x -k "ragged" --timeout 240 --timeout-method thread > $O/pytest_$n.txt 2>&1 || { tail -20 $O/pytest_$n.txt; exit 1; }
  echo "$n: $(tail -1 $O/pytest_$n.txt)"
done
cd /tmp
for r in 1 2; do
for lib in $R/multi-spectrogram-viewer_amd/lib/vd/*.so; do
  n=$(basename $lib .so)
  THESIA_LIB=$lib timeout -k 10 200 python3 $R/bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $O/b_${n}_$r.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$O/b_${n}_$r.log').read().strip().splitlines()[-1]); print('$r', '$n', 'display', round(d['roofline_display']['display_ms'], 3), 'step', round(d['ms_per_step'], 3))"
done
done
for lib in $R/multi-spectrogram-viewer_amd/lib/vd/*.so; do
  n=$(basename $lib .so)
  THESIA_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace -d $O/$n -o kt --output-format csv -- python3 $R/bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > $O/$n.log 2>&1 || exit $?
  python3 $R/scripts/kt_summary.py $n $O/$n/kt_kernel_trace.csv | grep -v 'stft\|range_init' || exit $?
done
