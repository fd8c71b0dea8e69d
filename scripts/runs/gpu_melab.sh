#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mel.py -x -q --timeout 120 --timeout-method thread > gpurun_out/melp_tests.log 2>&1 || { tail -30 gpurun_out/melp_tests.log; exit 1; }
tail -3 gpurun_out/melp_tests.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-c1 --no-e2e --no-rfft-roofline --mel-paths 1,2,3 > gpurun_out/melp_ab.log 2>&1 || { tail -20 gpurun_out/melp_ab.log; exit 1; }
cat gpurun_out/melp_ab.log | cut -c1-600
