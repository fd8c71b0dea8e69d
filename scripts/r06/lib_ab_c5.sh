#!/bin/bash
# A/B of a variant library against the product on the C5 line (conforming path), three
# interleaved rounds in separate processes: scripts/r06/lib_ab_c5.sh OUT VARIANT
# (multi-spectrogram-viewer_amd/lib/var/VARIANT.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r06_lib_ab}
V=$2
mkdir -p $O
for r in 1 2 3; do
  for v in product $V; do
    if [ $v = product ]; then unset THESIA_LIB; else export THESIA_LIB=$PWD/multi-spectrogram-viewer_amd/lib/var/$v.so; fi
    timeout -k 10 200 python bench.py --workload c5 --no-cpu-baseline > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err || { tail -5 $O/c5_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/c5_${v}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$r $v c5 step %.3f spec %.3f display %.3f' % (d['ms_per_step'], r['overlapped_ms'], d['roofline_display']['display_ms']), [round(b['kernel_ms'],3) for b in r['per_batch']])"
  done
done
