#!/bin/bash
# GPU suite + C5 bench (display A/B runs): stops at the first failure
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 2 > gpurun_out/bench_c5.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/bench_c5.log').read().strip().splitlines()[-1]); print('c5 ms/step', d['ms_per_step'], 'display_ms', d['roofline_display']['display_ms'])"
