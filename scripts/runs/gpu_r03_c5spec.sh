#!/bin/bash
# C5 spectrogram kernels: kernel A/B per n_fft on C5-shaped mono s16 amp-dB batches, and one SQ
# PMC pass over the C5 step's stft3 launches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r03_c5spec}
mkdir -p $O
export TMPDIR=/tmp
for nf in 256 512 1024 2048; do
  hop=$((nf / 4))
  timeout -k 10 200 python -u bench.py --channels 1 --input s16 --n-fft $nf --hop $hop --output amp_db --seconds 10 --sr 24000 --tracks 249 --kernels 2,3 --steps 5 --warmup 2 --no-cpu-baseline --no-c1 --no-e2e --no-rfft-roofline > $O/ab_$nf.log 2>&1 || exit $?
  grep kernels_ms $O/ab_$nf.log
done
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex "stft3" -d $O/pmc_sq -o p --output-format csv -- python3 $R/bench.py --workload c5 --steps 1 --warmup 1 > $O/pmc_sq.log 2>&1 || exit $?
echo done
