#!/bin/bash
# C5-shaped spectrogram batches (mono s16, amp dB rows, stft3): launch block count A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-s2_mb}; mkdir -p $O
NB="--no-cpu-baseline --no-c1 --no-e2e --no-rfft-roofline --steps 3 --warmup 1 --channels 1 --input s16 --output amp_db --seconds 10 --tracks 250 --kernel 3"
for cfg in "--sr 22050 --n-fft 256 --hop 64" "--sr 24000 --n-fft 512 --hop 128" "--sr 22050 --n-fft 1024 --hop 256" "--sr 24000 --n-fft 2048 --hop 512"; do
  timeout -k 10 200 python -u bench.py $cfg $NB --max-blocks 0,128,256,512,1024,2048 > $O/mb.log 2>&1 || exit $?
  echo "$cfg: $(grep max_blocks_ms $O/mb.log)"
done
