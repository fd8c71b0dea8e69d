#!/bin/bash
# A/B of variant libraries (scripts/build_variant.sh) on the C5 display step: for each round and
# each lib/var/*.so, one bench.py --workload c5 process. Prints name, step ms, display ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for lib in multi-spectrogram-viewer_amd/lib/var/*.so; do
    n=$(basename $lib .so)
    THESIA_LIB=$PWD/$lib timeout -k 10 180 python -u bench.py --workload c5 --steps 5 --warmup 1 \
      --no-cpu-baseline ${AB_ARGS:-} > gpurun_out/c5ab_$n.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/c5ab_$n.log').read().strip().splitlines()[-1]); print('$r', '$n', round(d['ms_per_step'], 3), round(d['roofline_display']['display_ms'], 3))"
  done
done
