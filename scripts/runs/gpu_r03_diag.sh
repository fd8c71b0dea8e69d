#!/bin/bash
# Round-3 diagnosis of the complex-output (window+rFFT) kernel's box-to-box spread: the memory
# pattern without arithmetic (row_pattern), the kernels 3 / 5 and row stores A/B with the box's
# own ceiling, the streaming tests, then FETCH / WRITE PMC passes of each kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r03_diag}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/microbench/row_pattern > $O/row_pattern.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --output complex --kernels 3,5 --row-stores 0,1,2 --no-cpu-baseline --no-c1 --no-e2e --steps 10 > $O/bench_complex.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --output power_db --kernels 3,5 --no-cpu-baseline --no-c1 --no-e2e --steps 10 > $O/bench_power.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-c1 --no-e2e --steps 10 > $O/bench_mel.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_streaming.py -x -q --timeout 120 --timeout-method thread > $O/pytest_streaming.log 2>&1 || exit $?
cd /tmp
for k in 3 5; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "stft" -d $O/pmc_k${k}_$c -o p --output-format csv -- python3 $R/bench.py --output complex --kernel $k --steps 2 --warmup 1 --no-cpu-baseline --no-c1 --no-e2e > $O/pmc_k${k}_$c.log 2>&1 || exit $?
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --output complex --kernels 3,5 --steps 5 --warmup 1 --no-cpu-baseline --no-c1 --no-e2e > $O/kt.log 2>&1 || exit $?
echo done
