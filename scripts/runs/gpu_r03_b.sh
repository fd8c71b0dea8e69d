#!/bin/bash
# Round 3: GPU suite, the viewer workload (benches/bench.rs entries) with a kernel trace, the
# stereo linear kinds' kernel A/B, and the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r03_b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 8 --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload viewer > $O/bench_viewer.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --output power_db --kernels 3,5 --no-cpu-baseline --no-c1 --no-e2e --no-rfft-roofline --steps 10 > $O/bench_power.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --output amp_db --kernels 3,5 --no-cpu-baseline --no-c1 --no-e2e --no-rfft-roofline --steps 10 > $O/bench_amp.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench_c4.log 2>&1 || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_viewer -o kt --output-format csv -- python3 $R/bench.py --workload viewer > $O/kt_viewer.log 2>&1 || exit $?
echo done
