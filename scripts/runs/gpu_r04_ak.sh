#!/bin/bash
# Round 4: stft3 vs stft5 at the 48 kHz viewer geometry (mel-128 dB, mono f32 and stereo) by batch
# size: where the streaming kernel with the heavier per-block setup starts to win.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_ak}
mkdir -p $O
for cfg in "1000 30 2" "100 30 2" "30 30 1" "10 30 1" "6 44 1" "2 30 1"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --win 1920 --hop 480 --n-fft 2048 --output mel_db --tracks $1 --seconds $2 --channels $3 --kernels 3,5 --steps 5 --warmup 2 > $O/v_$1_$2_$3.json 2> $O/v_$1_$2_$3.err || { tail -5 $O/v_$1_$2_$3.err; exit 1; }
  echo "tracks $1 seconds $2 channels $3: $(grep kernels_ms $O/v_$1_$2_$3.json | cut -c1-200)"
done
echo done
