#!/bin/bash
# Round 3: chunked fused display (intermediate reuse through the Infinity Cache): parity + A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r03_h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py -q -x -k "chunks or ragged" --timeout 200 --timeout-method thread > $O/pytest_chunks.txt 2>&1; rc=$?
tail -3 $O/pytest_chunks.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --workload c5 --steps 5 --warmup 2 --render-chunks 0,1024,256,128,64,32,16 > $O/bench_c5_chunks.log 2>&1 || exit $?
grep render_chunks $O/bench_c5_chunks.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_exact.py tests/test_gpu_multitrack.py -q -x --timeout 200 --timeout-method thread > $O/pytest_exact.txt 2>&1; rc=$?
tail -3 $O/pytest_exact.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload viewer > $O/bench_viewer.log 2>&1 || exit $?
echo done
