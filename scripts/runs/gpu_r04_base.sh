#!/bin/bash
# Round-4 baseline: C5 kernel trace (per display group) and FETCH / WRITE of the display passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_base}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --workload c5 --steps 2 --warmup 1"
timeout -k 10 240 python3 $B > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $B > $O/kt.log 2>&1 || exit $?
python3 $R/scripts/kt_summary.py c5 $O/kt/kt_kernel_trace.csv > $O/kt_summary.txt || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "grey_vert|resize_h" -d $O/pmc_fetch -o p --output-format csv -- python3 $B > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "grey_vert|resize_h" -d $O/pmc_write -o p --output-format csv -- python3 $B > $O/pmc_write.log 2>&1 || exit $?
echo done
