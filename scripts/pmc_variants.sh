set -u
cd "${GRAFT_REPO_ROOT}"
OUT=$PWD/gpurun_out; mkdir -p $OUT; REPO=$PWD
cd /tmp && export TMPDIR=/tmp
for v in 0 8 2; do
  THESIA_STFT_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU -d $OUT/pv_$v -o pmc --output-format csv -- python3 $REPO/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-rfft-roofline > $OUT/pv_$v.log 2>&1 || exit $?
done
