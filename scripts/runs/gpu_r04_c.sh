#!/bin/bash
# Round 4: the stripe display kernel's counters (serial groups), then the stft5 phase-ring A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_c}
mkdir -p $O
export TMPDIR=/tmp
export THESIA_RENDER_STREAMS=1
cd /tmp
B="$R/bench.py --workload c5 --steps 2 --warmup 1 --render-path 0"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $B > $O/kt.log 2>&1 || exit $?
python3 $R/scripts/kt_summary.py c5 $O/kt/kt_kernel_trace.csv > $O/kt_summary.txt || exit $?
cat $O/kt_summary.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex "stripe" -d $O/pmc_sq -o p --output-format csv -- python3 $B > $O/pmc_sq.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_BRANCH --kernel-include-regex "stripe" -d $O/pmc_lds -o p --output-format csv -- python3 $B > $O/pmc_lds.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "stripe" -d $O/pmc_fetch -o p --output-format csv -- python3 $B > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "stripe" -d $O/pmc_write -o p --output-format csv -- python3 $B > $O/pmc_write.log 2>&1 || exit $?
cd $R
EXP=$R/multi-spectrogram-viewer_amd/lib/libthesia_exp.so
THESIA_LIB=$EXP timeout -k 10 200 python3 scripts/check_variant.py 1 > $O/variant1_parity.txt 2>&1; rc=$?
cat $O/variant1_parity.txt
if [ $rc -eq 0 ]; then
  THESIA_LIB=$EXP timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --variants 0,1 > $O/bench_c4_variants.json 2> $O/bench_c4_variants.err || exit $?
  grep variants_kernel_ms $O/bench_c4_variants.json
fi
echo done
