#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
THESIA_LIB=$PWD/multi-spectrogram-viewer_amd/lib/vd/wv12.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_configs.py tests/test_gpu_streaming.py tests/test_gpu_stft.py > gpurun_out/wv12_tests.log 2>&1
rc=$?; tail -3 gpurun_out/wv12_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/runs/gpu_vd_ab.sh
