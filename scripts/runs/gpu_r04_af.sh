#!/bin/bash
# Round 4: host gap between the C5 phases after trimming the range path (no device-wide sync,
# numpy reductions, no all_reduce on one rank): C5 line twice and a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_af}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
timeout -k 10 300 python3 bench.py --workload c5 --steps 10 --warmup 2 > $O/bench_c5_$r.json 2> $O/bench_c5_$r.err || { tail -20 $O/bench_c5_$r.err; exit 1; }
tail -1 $O/bench_c5_$r.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['roofline_display']['display_ms'], d['roofline']['overlapped_ms'])"
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --workload c5 --steps 5 --warmup 1 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 $R/scripts/kt_gaps.py $O/kt/kt_kernel_trace.csv
echo done
