#!/bin/bash
# stft2 (kernel 2, the general-geometry kernel) builds A/B via THESIA_LIB (lib/vd/*.so),
# alternating rounds in separate processes, forced kernel 2 on three shapes
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${1:-stft2_ab}; mkdir -p $O
COMMON="--no-cpu-baseline --no-e2e --no-rfft-roofline --no-c1 --steps 5 --warmup 1 --kernel 2"
for r in $(seq ${ROUNDS:-2}); do
for lib in $R/multi-spectrogram-viewer_amd/lib/vd/*.so; do
  n=$(basename $lib .so)
  i=0
  for cfg in "--output complex" "--tracks 1000 --seconds 10 --sr 24000 --channels 1 --input s16 --n-fft 1024 --hop 256 --output complex" "--sr 44100 --n-fft 2048 --win 1764 --hop 441 --channels 1 --input s16 --output mel_db --n-mels 0"; do
    i=$((i+1))
    THESIA_LIB=$lib timeout -k 10 200 python3 bench.py $cfg $COMMON > $O/${n}_${i}_$r.log 2>&1 || exit $?
    python3 -c "import json; d=json.loads(open('$O/${n}_${i}_$r.log').read().strip().splitlines()[-1]); print('$r $n cfg$i', round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],3), d['roofline']['kernel'][:24])"
  done
done
done
