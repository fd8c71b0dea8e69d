#!/bin/bash
# display path A/B on C5 (render paths 0 / 5) + the render tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r03_disp}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -q --timeout 300 --timeout-method thread -k "ragged" > $O/pytest_render.txt 2>&1; rc=$?
tail -2 $O/pytest_render.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --render-paths 0,5 > $O/bench_c5.log 2>&1 || exit $?
grep render_paths $O/bench_c5.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_p5 -o kt --output-format csv -- python3 $R/bench.py --workload c5 --steps 2 --warmup 1 --render-path 5 > $O/kt_p5.log 2>&1 || exit $?
echo done
