#!/bin/bash
# Round 4, first call: the changed GPU tests (C2 direct bounds, library pool), then the C5 baseline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_a}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_configs.py::test_c2_six_sample_rates_power_db tests/test_gpu_multitrack.py tests/test_gpu_napi.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
grep "C2 \|passed\|failed" $O/pytest.txt
bash $R/scripts/runs/gpu_r04_base.sh ${1:-r04_a}
