#!/bin/bash
# Round 4: render parity tests (paths 0..4, incl. the 9 / 10-accumulator stripe instances), the
# per-group display at the C5 geometry (path 0 and kernel trace), the C5 line with the batches
# policies 0 / 2 (concurrent vs serial spectrogram batches).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_s}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py -k "render or c5" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
cd /tmp
THESIA_RENDER_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktg -o kt --output-format csv -- python3 $R/scripts/display_groups_ab.py 0 > $O/ktg.log 2>&1 || { tail -5 $O/ktg.log; exit 1; }
python3 $R/scripts/kt_segments.py $O/ktg/kt_kernel_trace.csv > $O/groups_kt0.txt
cat $O/groups_kt0.txt
timeout -k 10 300 python3 $R/bench.py --workload c5 --steps 10 --warmup 2 --spec-policies 0,2 --render-paths 0,3 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
grep render_paths $O/bench_c5.json
tail -1 $O/bench_c5.json | python3 -c "import json,sys; d=json.load(sys.stdin); r=d['roofline']; print(d['ms_per_step'], d['roofline_display']['display_ms'], r['overlapped_ms'], r['kernel_ms'], r['batches_policy_ms'])"
echo done
