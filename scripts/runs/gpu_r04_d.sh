#!/bin/bash
# Round 4: stripe kernel v2 -- render parity tests, per-group A/B, C5 line with render paths 0/3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_d}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py -k "render or c5" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
cd /tmp
THESIA_RENDER_STREAMS=1 timeout -k 10 400 python3 $R/scripts/display_groups_ab.py 0,3 > $O/groups_ab.txt 2>&1 || { tail $O/groups_ab.txt; exit 1; }
tail -1 $O/groups_ab.txt
timeout -k 10 300 python3 $R/bench.py --workload c5 --steps 10 --warmup 2 --render-paths 0,3 --spec-policies 0,1 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
grep render_paths $O/bench_c5.json
tail -1 $O/bench_c5.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['roofline_display']['display_ms'], d['roofline']['overlapped_ms'], d['roofline']['batches_policy_ms'])"
echo done
