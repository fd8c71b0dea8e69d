#!/bin/bash
# Round 4: experiment-build display A/B: THESIA_HNB=8 (8 row buffers in the horizontal DMA pass for
# one-chunk spans) against the default, per group alone and on the C5 line (two rounds each).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_u}
mkdir -p $O
export TMPDIR=/tmp
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
run_cfg base THESIA_HNB=4 || exit 1
run_cfg hnb8 THESIA_HNB=8 || exit 1
run_cfg base2 THESIA_HNB=4 || exit 1
run_cfg hnb8_2 THESIA_HNB=8 || exit 1
echo done
