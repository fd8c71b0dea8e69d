#!/bin/bash
# GPU suite, then the C5 line with the display A/B of render paths 0 / 3 (5 interleaved rounds,
# one process) and the C5 spectrogram kernels' trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${1:-s2_check}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
tail -3 $O/pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --render-paths 0,3 > $O/bench_c5.log 2>&1 || exit $?
grep render_paths $O/bench_c5.log
python3 -c "import json; d=json.loads(open('$O/bench_c5.log').read().strip().splitlines()[-1]); print('step', d['ms_per_step'], 'spec kernels', d['roofline']['kernel_ms'], 'overlapped', d['roofline']['overlapped_ms'], 'display', d['roofline_display']['display_ms'])"
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1 || exit $?
python3 $R/scripts/kt_summary.py c5 $O/kt/kt_kernel_trace.csv
