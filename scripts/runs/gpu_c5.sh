#!/bin/bash
# C5 display path: GPU parity of the render tests, then the C5 bench with the batched render
# (default) and with per-track launches (THESIA_RENDER_PER_TRACK=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 > gpurun_out/c5_batch.log 2>&1
rc=$?; echo "c5 batch rc=$rc"; tail -1 gpurun_out/c5_batch.log; [ $rc -ne 0 ] && exit $rc
THESIA_RENDER_PER_TRACK=1 timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 > gpurun_out/c5_pertrack.log 2>&1
rc=$?; echo "c5 per-track rc=$rc"; tail -1 gpurun_out/c5_pertrack.log
exit $rc
