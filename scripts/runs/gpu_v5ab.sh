#!/bin/bash
# A/B of stft5 variant libraries (scripts/build_v5.sh) on the C4 shard: for each round and each
# lib/v5/*.so, one bench.py process (kernel 5, HIP-event kernel time). Prints name + kernel_ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for lib in multi-spectrogram-viewer_amd/lib/v5/*.so; do
    n=$(basename $lib .so)
    THESIA_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --kernel 5 --steps 10 --warmup 2 \
      --no-cpu-baseline --no-c1 --no-rfft-roofline ${V5_ARGS:-} > gpurun_out/v5_$n.log 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/v5_$n.log').read().strip().splitlines()[-1]); print('$r', '$n', round(d['roofline']['kernel_ms'], 4))"
  done
done
