#!/bin/bash
# Round 4: per-group display A/B (paths 0/3/4) and per-group kernel trace (path 0) at the C5 step's
# geometry (up_ratio against 48 kHz), then counters of group 10's two-pass kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_p}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
THESIA_RENDER_STREAMS=1 timeout -k 10 400 python3 $R/scripts/display_groups_ab.py 0,3,4 > $O/groups_ab.txt 2>&1 || { tail $O/groups_ab.txt; exit 1; }
tail -1 $O/groups_ab.txt
THESIA_RENDER_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktg -o kt --output-format csv -- python3 $R/scripts/display_groups_ab.py 0 > $O/ktg.log 2>&1 || { tail -5 $O/ktg.log; exit 1; }
python3 $R/scripts/kt_segments.py $O/ktg/kt_kernel_trace.csv > $O/groups_kt0.txt
cat $O/groups_kt0.txt
cd $R
bash scripts/runs/gpu_r04_m.sh ${1:-r04_p}/m10 10 0 "grey_vert|resize_h"
