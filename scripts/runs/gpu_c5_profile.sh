#!/bin/bash
# C5 step profile: kernel trace (per-launch durations of the 4 spectrogram batches and the
# display launches), then one SQ pass and FETCH / WRITE passes over the spectrogram launches.
# Usage: gpu_c5_profile.sh OUTDIR_NAME
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-c5prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --workload c5 --steps 2 --warmup 1"
[ "${SKIP_KT:-0}" = 1 ] || timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $B > $O/kt.log 2>&1 || exit $?
[ "${SKIP_KT:-0}" = 1 ] || python3 $R/scripts/kt_summary.py c5 $O/kt/kt_kernel_trace.csv > $O/kt_summary.txt || exit $?
cat $O/kt_summary.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex "stft" -d $O/pmc_sq -o p --output-format csv -- python3 $B > $O/pmc_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "stft" -d $O/pmc_fetch -o p --output-format csv -- python3 $B > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "stft" -d $O/pmc_write -o p --output-format csv -- python3 $B > $O/pmc_write.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-include-regex "grey_vert|resize_h" -d $O/pmc_dsq -o p --output-format csv -- python3 $B > $O/pmc_dsq.log 2>&1 || exit $?
echo done
