#!/bin/bash
# Parity of one stft5 variant library (scripts/build_v5.sh) on the stft5 tests, then the A/B of
# every lib/v5/*.so (scripts/runs/gpu_v5ab.sh). Usage: V5=name bash scripts/runs/gpu_v5par.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
THESIA_LIB=$PWD/multi-spectrogram-viewer_amd/lib/v5/${V5}.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_mel.py tests/test_gpu_parity.py -k "(128 and kernels_own) or bench or track_edges" > gpurun_out/v5par_${V5}.log 2>&1
rc=$?; tail -4 gpurun_out/v5par_${V5}.log; [ $rc -eq 0 ] || exit $rc
bash scripts/runs/gpu_v5ab.sh
