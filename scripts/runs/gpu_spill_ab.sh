#!/bin/bash
# stft3 with / without the spilled loop invariants (lib/vd/*.so via THESIA_LIB), alternating
# rounds in separate processes: the C4 line's window+rFFT kernel (stft3 complex, n_fft 2048),
# an n_fft 1024 int16-mono amp-dB launch, and the C5 step's spectrogram batches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${1:-spill_ab}; mkdir -p $O
for r in $(seq ${ROUNDS:-2}); do
for lib in $R/multi-spectrogram-viewer_amd/lib/vd/*.so; do
  n=$(basename $lib .so)
  THESIA_LIB=$lib timeout -k 10 200 python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-c1 > $O/c4_${n}_$r.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$O/c4_${n}_$r.log').read().strip().splitlines()[-1]); w=d['roofline_window_rfft']; print('$r $n c4 mel', round(d['roofline']['kernel_ms'],3), 'rfft', round(w['kernel_ms'],3), round(w['frac'],3))"
  THESIA_LIB=$lib timeout -k 10 200 python3 bench.py --tracks 1000 --seconds 10 --sr 24000 --channels 1 --input s16 --n-fft 1024 --hop 256 --output amp_db --no-cpu-baseline --no-e2e --no-rfft-roofline --no-c1 --steps 5 --warmup 1 > $O/n1024_${n}_$r.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$O/n1024_${n}_$r.log').read().strip().splitlines()[-1]); print('$r $n n1024 amp dB', round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],3))"
  THESIA_LIB=$lib timeout -k 10 200 python3 bench.py --workload c5 --steps 20 --warmup 2 --no-cpu-baseline > $O/c5_${n}_$r.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$O/c5_${n}_$r.log').read().strip().splitlines()[-1]); print('$r $n c5 step', round(d['ms_per_step'],3), 'spec', round(d['roofline']['overlapped_ms'],3), [round(b['kernel_ms'],3) for b in d['roofline']['per_batch']])"
done
done
