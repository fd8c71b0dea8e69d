#!/bin/bash
# PMC passes over the C5 step (display kernels): one counter set per run.
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; REPO=$PWD
cd /tmp && export TMPDIR=/tmp
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/pc5_$i -o pmc --output-format csv -- python3 $REPO/bench.py --workload c5 --steps 1 --warmup 1 > $OUT/pc5_$i.log 2>&1 || exit $?
  echo "done $c"; i=$((i+1))
done
