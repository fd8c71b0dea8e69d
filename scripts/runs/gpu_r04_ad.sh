#!/bin/bash
# Round 4: stft5 scheduler-flag variants (lib/libthesia_v{t,mc,il}.so: AMDGPU trackers, max-memory-
# clause, max-ilp strategies on stft5_kernels.hip only) vs the default build, C4 line, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_ad}
mkdir -p $O
for r in 1 2 3; do
  for v in def t mc il; do
    L=$R/multi-spectrogram-viewer_amd/lib/libthesia.so; [ $v != def ] && L=$R/multi-spectrogram-viewer_amd/lib/libthesia_v$v.so
    THESIA_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/c4_${v}_$r.json 2> $O/c4_${v}_$r.err || { tail -5 $O/c4_${v}_$r.err; exit 1; }
    tail -1 $O/c4_${v}_$r.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$v', $r, round(d['ms_per_step'],3))"
  done
done
echo done
