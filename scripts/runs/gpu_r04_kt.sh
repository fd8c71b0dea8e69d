#!/bin/bash
# Round 4 final: rocprofv3 kernel-trace summaries of the default bench line (C4) and the C5 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_kt}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c4 -o kt --output-format csv -- python3 $R/bench.py > $O/c4.log 2>&1 || { tail -5 $O/c4.log; exit 1; }
tail -1 $O/c4.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5 -o kt --output-format csv -- python3 $R/bench.py --workload c5 --steps 10 --warmup 2 > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
tail -1 $O/c5.log | cut -c1-300
echo done
