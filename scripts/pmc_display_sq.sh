#!/bin/bash
# SQ counters of the display kernels over the C5 bench (one pass)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/pmc_dsq; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-include-regex "grey_vert|resize_h" -d $O -o p --output-format csv -- python3 $R/bench.py --workload c5 --steps 1 --warmup 1 > $O/run.log 2>&1 || exit $?
echo done
