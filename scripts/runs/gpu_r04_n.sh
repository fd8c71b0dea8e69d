#!/bin/bash
# Round 4: render parity tests (paths 0..4), per-group A/B of paths 0/3/4, the C5 line, kernel traces
# A/B of paths 0/3/4, the C5 line, and a kernel trace of the C5 bench (per-kernel display times).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_n}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py -k "render or c5" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
cd /tmp
THESIA_RENDER_STREAMS=1 timeout -k 10 400 python3 $R/scripts/display_groups_ab.py 0,3,4 > $O/groups_ab.txt 2>&1 || { tail $O/groups_ab.txt; exit 1; }
tail -1 $O/groups_ab.txt
timeout -k 10 300 python3 $R/bench.py --workload c5 --steps 10 --warmup 2 --render-paths 0,3,4 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
grep render_paths $O/bench_c5.json
tail -1 $O/bench_c5.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['roofline_display']['display_ms'], d['roofline']['overlapped_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python3 $R/bench.py --workload c5 --steps 5 --warmup 1 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python3 $R/scripts/kt_summary.py c5 $O/kt/kt_kernel_trace.csv > $O/kt_summary.txt
cat $O/kt_summary.txt

THESIA_RENDER_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktg -o kt --output-format csv -- python3 $R/scripts/display_groups_ab.py 0 > $O/ktg.log 2>&1 || { tail -5 $O/ktg.log; exit 1; }
python3 $R/scripts/kt_segments.py $O/ktg/kt_kernel_trace.csv > $O/groups_kt0.txt
cat $O/groups_kt0.txt
echo done
