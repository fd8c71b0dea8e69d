#!/bin/bash
# Kernel-trace A/B of variant libraries (scripts/build_variant.sh) on the C5 display step: one
# rocprofv3 --kernel-trace run of bench.py --workload c5 per lib/var/*.so; prints per-kernel
# time per step (tools: scripts/kt_summary.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in multi-spectrogram-viewer_amd/lib/var/*.so; do
  n=$(basename $lib .so)
  (cd /tmp && THESIA_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/kt_$n -o kt \
    --output-format csv -- python3 $R/bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline \
    > $R/gpurun_out/kt_$n.log 2>&1) || exit $?
  python3 scripts/kt_summary.py $n gpurun_out/kt_$n/kt_kernel_trace.csv
done
