#!/bin/bash
# A/B of display variant libraries (scripts/build_variant_display.sh): C5 display_ms per library,
# two interleaved rounds, one bench process each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for lib in multi-spectrogram-viewer_amd/lib/vd/*.so; do
    n=$(basename $lib .so)
    THESIA_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --workload c5 --steps 2 --warmup 1 > gpurun_out/vd_$n.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/vd_$n.log').read().strip().splitlines()[-1]); print('$r', '$n', 'display', round(d['roofline_display']['display_ms'], 3), 'step', round(d['ms_per_step'], 3), 'spec_kernels', round(d['roofline']['kernel_ms'], 3))"
  done
done
