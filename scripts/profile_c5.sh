#!/bin/bash
# C5 display evidence: kernel trace of bench --workload c5, then FETCH_SIZE / WRITE_SIZE passes
# (separate runs) restricted to the display kernels. Output: gpurun_out/$1/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${1:-c5prof}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --workload c5 --steps 3 --warmup 1 > $O/kt.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "grey_vert|resize_h|minmax" -d $O/pmc_$c -o p --output-format csv -- python3 $R/bench.py --workload c5 --steps 1 --warmup 1 > $O/pmc_$c.log 2>&1 || exit $?
done
echo done
