#!/bin/bash
# Round 4: the silent-track render tests (GreyMap fallback branch, zero span) and the ragged groups.
set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/r04_as
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -x -q -k "silent or ragged" --timeout 240 --timeout-method thread > gpurun_out/r04_as/pytest.txt 2>&1; rc=$?; tail -15 gpurun_out/r04_as/pytest.txt; exit $rc
