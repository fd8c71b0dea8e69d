#!/bin/bash
# Round 4 check: the whole GPU suite, smoke, the default bench line (C4) and the C5 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_w}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -30 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('C4', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
tail -1 $O/bench_c5.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('C5', d['ms_per_step'], d['roofline_display']['display_ms'], d['roofline_display']['traffic'], d['roofline_display_valu_issue']['frac'])"
echo done
