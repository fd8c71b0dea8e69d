#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_spec_streams.py > gpurun_out/spec_ab.log 2>&1 || { tail -20 gpurun_out/spec_ab.log; exit 1; }
tail -1 gpurun_out/spec_ab.log
bash scripts/runs/gpu_quick.sh
