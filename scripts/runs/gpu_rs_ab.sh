#!/bin/bash
# Display groups in flight at once (THESIA_RENDER_STREAMS 1 vs 4): the render tests on the
# default, then C5 steps alternating the two settings in separate processes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${1:-rs_ab}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -q -x -k "render or ragged or image" --timeout 240 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -20 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in $(seq ${ROUNDS:-3}); do
for ns in 1 4; do
  THESIA_RENDER_STREAMS=$ns timeout -k 10 200 python3 bench.py --workload c5 --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > $O/b_${ns}_$r.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$O/b_${ns}_$r.log').read().strip().splitlines()[-1]); print('$r', 'streams $ns', 'display', round(d['roofline_display']['display_ms'], 3), 'step', round(d['ms_per_step'], 3))"
done
done
