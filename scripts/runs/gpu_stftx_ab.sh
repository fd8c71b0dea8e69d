#!/bin/bash
# stftx builds (lib/vd/*.so via THESIA_LIB): the bit-exact tests on each, then the viewer line's
# kernel times behind add_tracks in alternating rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/${1:-stftx_ab}; mkdir -p $O
for lib in $R/multi-spectrogram-viewer_amd/lib/vd/*.so; do
  n=$(basename $lib .so)
  THESIA_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_exact.py -q -x --timeout 120 --timeout-method thread > $O/pytest_$n.txt 2>&1 || { tail -20 $O/pytest_$n.txt; exit 1; }
  echo "$n: $(tail -1 $O/pytest_$n.txt)"
done
for r in $(seq ${ROUNDS:-2}); do
for lib in $R/multi-spectrogram-viewer_amd/lib/vd/*.so; do
  n=$(basename $lib .so)
  THESIA_LIB=$lib timeout -k 10 300 python3 bench.py --workload viewer > $O/v_${n}_$r.log 2>&1 || exit $?
  python3 -c "
import json; d=json.loads(open('$O/v_${n}_$r.log').read().strip().splitlines()[-1]); e=d['entries']
print('$r $n', 'stftx', round(e['add_tracks_kernels']['stftx']['kernel_ms'],4), 'melspec stftx', round(e['get_melspectrogram']['stftx (reference order, bit-exact)']['kernel_ms'],4), 'add_tracks', round(e['add_tracks']['gpu_ms'],3))"
done
done
