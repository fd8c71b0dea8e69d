#!/bin/bash
# Round 4: render parity, per group alone (path 0), C5 line twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_ac}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py -k "render or c5" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
cd /tmp
THESIA_RENDER_STREAMS=1 timeout -k 10 300 python3 $R/scripts/display_groups_ab.py 0 > $O/groups.txt 2>&1 || { tail $O/groups.txt; exit 1; }
tail -1 $O/groups.txt
cd $R
for r in 1 2; do
timeout -k 10 300 python3 bench.py --workload c5 --steps 10 --warmup 2 --render-paths 0 > $O/bench_c5_$r.json 2> $O/bench_c5_$r.err || { tail -20 $O/bench_c5_$r.err; exit 1; }
grep render_paths $O/bench_c5_$r.json
tail -1 $O/bench_c5_$r.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['roofline_display']['display_ms'])"
done
echo done
