#!/bin/bash
# GPU parity, then A/B of the stft3 wave-priority phases (default) vs none (variant 4096) for
# the mel, complex and power-dB kinds, then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for o in mel_db complex power_db; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-rfft-roofline --output $o --variants 0,4096 > gpurun_out/prio_$o.log 2>&1
  rc=$?; echo "ab $o rc=$rc"; grep variants gpurun_out/prio_$o.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.log
exit $rc
