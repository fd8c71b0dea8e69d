#!/bin/bash
# wide vertical pass: ragged-group byte tests on path 3, C5 display A/B paths 0 / 3, and LDS
# bank-conflict counters of the display kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${1:-s2_wide}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -q -x -k "ragged" --timeout 240 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --render-paths 0,3 > $O/ab.log 2>&1 || exit $?
grep render_paths $O/ab.log
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex "grey_vert|resize_h" -d $O/pmc_lds -o p --output-format csv -- python3 $R/bench.py --workload c5 --steps 1 --warmup 1 --render-path 3 > $O/pmc_lds.log 2>&1 || exit $?
python3 $R/scripts/pmc_summary.py $O/pmc_lds/p_counter_collection.csv
cd $R
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- python3 bench.py --workload c5 --steps 2 --warmup 1 --render-path 3 > $O/kt.log 2>&1 || exit $?
python3 scripts/kt_summary.py p3 $O/kt/kt_kernel_trace.csv | grep -v 'stft\|range_init'
