#!/bin/bash
# Round 3: GPU suite, viewer + C4 + C5 lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r03_e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 8 --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload viewer > $O/bench_viewer.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench_c4.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload c5 > $O/bench_c5.log 2>&1 || exit $?
echo done
