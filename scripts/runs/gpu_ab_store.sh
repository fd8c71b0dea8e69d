#!/bin/bash
# A/B of the LDS-staged 16-byte row stores (default) vs lane-wise stores (variant 1024) for the
# complex and power-dB kinds, after the GPU parity suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for o in complex power_db amp_db; do
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-rfft-roofline --output $o --variants 0,1024 > gpurun_out/ab_$o.log 2>&1
  rc=$?; echo "ab $o rc=$rc"; grep variants gpurun_out/ab_$o.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.log
exit $rc
