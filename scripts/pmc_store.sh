#!/bin/bash
# HBM write/fetch traffic of the complex- and power-dB-output kernels with LDS-staged 16-byte
# row stores (variant 0) and lane-wise stores (variant 1024). One counter set per run.
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; REPO=$PWD
cd /tmp && export TMPDIR=/tmp
for o in complex power_db; do
  for v in 0 1024; do
    for c in WRITE_SIZE FETCH_SIZE; do
      THESIA_STFT_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/ps_${o}_${v}_$c -o pmc --output-format csv -- python3 $REPO/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rfft-roofline --output $o > $OUT/ps_${o}_${v}_$c.log 2>&1 || exit $?
      echo "done $o $v $c"
    done
  done
done
