#!/bin/bash
# C5 steps with HIP's hardware queues per process at 4 (the box's default) vs 8: the library's
# stream pool (4 streams) plus the caller's and the library's default stream exceed 4 queues
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=$PWD/gpurun_out/${1:-hwq_ab}; mkdir -p $O
for r in $(seq ${ROUNDS:-3}); do
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --workload c5 --steps 20 --warmup 2 --no-cpu-baseline > $O/b_${q}_$r.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$O/b_${q}_$r.log').read().strip().splitlines()[-1]); print('$r', 'hwq $q', 'display', round(d['roofline_display']['display_ms'], 3), 'spec', round(d['roofline']['overlapped_ms'], 3), 'step', round(d['ms_per_step'], 3))"
done
done
cd /tmp
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/kt8 -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/kt8.log 2>&1
