#!/bin/bash
# Round 3: stft6 parity + in-process A/B vs stft5 (C4 shard) + kernel trace, then the GPU suite,
# viewer / C4 / C5 lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r03_f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stft6.py -q -x --timeout 200 --timeout-method thread > $O/pytest_stft6.txt 2>&1; rc=$?
tail -3 $O/pytest_stft6.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --kernels 5,6 --no-cpu-baseline --no-e2e --no-c1 > $O/bench_ab56.log 2>&1 || exit $?
grep kernels_ms $O/bench_ab56.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt6 -o kt -- python3 -u bench.py --steps 5 --warmup 2 --kernel 6 --no-cpu-baseline --no-e2e --no-c1 --no-rfft-roofline > $O/bench_k6_prof.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 8 --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload viewer > $O/bench_viewer.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload c5 > $O/bench_c5.log 2>&1 || exit $?
echo done
