#!/bin/bash
# Round 4: display A/Bs on the experiment build (per group alone and on the C5 line): the
# grey_vert staging (THESIA_VSTAGE), its tile-row cap (THESIA_VROWS_CAP), two frames per lane for
# the downsampling groups (THESIA_VFPL2), two rows per barrier in the horizontal pass
# (THESIA_HRP); render parity tests of the product build first; then the per-batch max-blocks A/B.
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
run_cfg() {  # name, env assignments
  local name=$1; shift
  env THESIA_LIB=$R/multi-spectrogram-viewer_amd/lib/libthesia_exp.so THESIA_RENDER_STREAMS=1 "$@" \
    timeout -k 10 300 python3 $R/scripts/display_groups_ab.py 0 > $O/groups_$name.txt 2>&1 || { tail $O/groups_$name.txt; return 1; }
  echo "$name: $(tail -1 $O/groups_$name.txt)"
  env THESIA_LIB=$R/multi-spectrogram-viewer_amd/lib/libthesia_exp.so "$@" \
    timeout -k 10 300 python3 $R/bench.py --workload c5 --steps 10 --warmup 2 > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; return 1; }
  tail -1 $O/bench_$name.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$name c5', d['ms_per_step'], d['roofline_display']['display_ms'])"
}
run_cfg base THESIA_VSTAGE=1 || exit 1
run_cfg vstage0 THESIA_VSTAGE=0 || exit 1
run_cfg hrp2 THESIA_HRP=2 || exit 1
run_cfg fpl2 THESIA_VFPL2=1 || exit 1
run_cfg cap192 THESIA_VROWS_CAP=192 || exit 1
run_cfg cap256 THESIA_VROWS_CAP=256 || exit 1
timeout -k 10 300 python3 $R/bench.py --workload c5 --steps 10 --warmup 2 --max-blocks 0,64,128,192,512 > $O/bench_mb.json 2> $O/bench_mb.err || { tail -20 $O/bench_mb.err; exit 1; }
tail -1 $O/bench_mb.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['roofline']['per_batch_max_blocks_ms'], d['roofline']['per_batch'])"
echo done
