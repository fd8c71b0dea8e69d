#!/bin/bash
# Round-end evidence on one GPU box: GPU test suite, the default bench line (C4), the C5, viewer
# and C3 lines, a kernel trace of the default bench, separate PMC passes (HBM traffic; SQ mix) of its
# launches. Output: gpurun_out/$1/ (copy what is judged into profiles/$1/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.txt 2>&1 || exit $?
timeout -k 10 600 python bench.py > $O/bench_c4.log 2>&1 || exit $?
grep '^{' $O/bench_c4.log | tail -1 > $O/bench_c4.json
timeout -k 10 300 python bench.py --workload c5 > $O/bench_c5.log 2>&1 || exit $?
grep '^{' $O/bench_c5.log | tail -1 > $O/bench_c5.json
timeout -k 10 300 python bench.py --workload viewer > $O/bench_viewer.log 2>&1 || exit $?
grep '^{' $O/bench_viewer.log | tail -1 > $O/bench_viewer.json
timeout -k 10 300 python bench.py --workload c3 --no-cpu-baseline --no-e2e > $O/bench_c3.log 2>&1 || exit $?
grep '^{' $O/bench_c3.log | tail -1 > $O/bench_c3.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-c1 --no-e2e > $O/kt.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "stft5|stft3" -d $O/pmc_fetch -o p --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c1 --no-e2e --no-rfft-roofline > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "stft5|stft3" -d $O/pmc_write -o p --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c1 --no-e2e --no-rfft-roofline > $O/pmc_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex "stft5" -d $O/pmc_sq -o p --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-c1 --no-e2e --no-rfft-roofline > $O/pmc_sq.log 2>&1 || exit $?
echo done
