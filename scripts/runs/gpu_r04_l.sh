#!/bin/bash
# Round 4: display kernels per C5 group alone (one stream), kernel trace, render path 0 and 3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_l}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for p in ${2:-0 3}; do
THESIA_RENDER_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt$p -o kt --output-format csv -- python3 $R/scripts/display_groups_ab.py $p > $O/kt$p.log 2>&1 || { tail -5 $O/kt$p.log; exit 1; }
python3 $R/scripts/kt_groups.py $O/kt$p/kt_kernel_trace.csv > $O/groups_kt$p.txt
cat $O/groups_kt$p.txt
done
echo done
