#!/bin/bash
# Round 3: GPU suite, then the C5 line and a kernel trace of it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r03_c5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 8 --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --render-paths 0,5 > $O/bench_c5.log 2>&1 || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_c5 -o kt --output-format csv -- python3 $R/bench.py --workload c5 --steps 3 --warmup 1 > $O/kt_c5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_c5_p5 -o kt --output-format csv -- python3 $R/bench.py --workload c5 --steps 3 --warmup 1 --render-path 5 > $O/kt_c5_p5.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --runtime-trace --stats -d $O/rt_viewer -o rt --output-format csv -- python3 $R/bench.py --workload viewer > $O/rt_viewer.log 2>&1 || exit $?
echo done
