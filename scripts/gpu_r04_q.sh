#!/bin/bash
# Round 4: grey_vert staging A/B (THESIA_VSTAGE 0/1) and tile-row cap A/B (THESIA_VROWS_CAP) on the
# experiment build, per group and on the C5 line; then render parity tests of the product build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_q}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py -k "render or c5" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
cd /tmp
export THESIA_LIB=$R/multi-spectrogram-viewer_amd/lib/libthesia_exp.so
for cfg in "1 128" "0 128" "1 192" "1 256"; do
  set -- $cfg
  THESIA_VSTAGE=$1 THESIA_VROWS_CAP=$2 THESIA_RENDER_STREAMS=1 timeout -k 10 300 python3 $R/scripts/display_groups_ab.py 0 > $O/groups_$1_$2.txt 2>&1 || { tail $O/groups_$1_$2.txt; exit 1; }
  echo "vstage $1 cap $2: $(tail -1 $O/groups_$1_$2.txt)"
  THESIA_VSTAGE=$1 THESIA_VROWS_CAP=$2 timeout -k 10 300 python3 $R/bench.py --workload c5 --steps 10 --warmup 2 > $O/bench_$1_$2.json 2> $O/bench_$1_$2.err || { tail -20 $O/bench_$1_$2.err; exit 1; }
  tail -1 $O/bench_$1_$2.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('c5', d['ms_per_step'], d['roofline_display']['display_ms'])"
done
unset THESIA_LIB
timeout -k 10 300 python3 $R/bench.py --workload c5 --steps 10 --warmup 2 --max-blocks 0,64,128,192,512 > $O/bench_mb.json 2> $O/bench_mb.err || { tail -20 $O/bench_mb.err; exit 1; }
tail -1 $O/bench_mb.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d[\"roofline\"][\"per_batch_max_blocks_ms\"], d[\"roofline\"][\"per_batch\"])"
echo done
