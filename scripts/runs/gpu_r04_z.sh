#!/bin/bash
# Round 4: the canonical C4 line with the previous stft5 (lib/libthesia_ab.so: HEAD's stft5 object)
# vs the viewer-rule stft5 (lib/libthesia.so), interleaved, three rounds each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_z}
mkdir -p $O
for r in 1 2 3; do
  for lib in ab cur; do
    L=$R/multi-spectrogram-viewer_amd/lib/libthesia.so; [ $lib = ab ] && L=$R/multi-spectrogram-viewer_amd/lib/libthesia_ab.so
    THESIA_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 3 > $O/c4_${lib}_$r.json 2> $O/c4_${lib}_$r.err || { tail -5 $O/c4_${lib}_$r.err; exit 1; }
    tail -1 $O/c4_${lib}_$r.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$lib', $r, round(d['ms_per_step'],3))"
  done
done
echo done
