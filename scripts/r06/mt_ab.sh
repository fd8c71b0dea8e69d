#!/bin/bash
# A/B of add_tracks' copy stream: the product library against lib/var/mtprev.so
# (the same sources with the uploads on the library stream), three interleaved rounds of the
# viewer line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r06_mt_ab}
mkdir -p $O
for r in 1 2 3; do
  for v in product mtprev; do
    if [ $v = mtprev ]; then export THESIA_LIB=$PWD/multi-spectrogram-viewer_amd/lib/var/mtprev.so; else unset THESIA_LIB; fi
    timeout -k 10 200 python bench.py --workload viewer > $O/viewer_${v}_$r.json 2> $O/viewer_${v}_$r.err || { tail -5 $O/viewer_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/viewer_${v}_$r.json').read().strip().splitlines()[-1]); e=d['entries']
print('$r $v add_tracks %.3f get_spec_image %.3f' % (e['add_tracks']['gpu_ms'], e['get_spec_image']['gpu_ms']))"
  done
done
