#!/bin/bash
# A/B of stftq's LDS swizzles: the product library against lib/var/preswz.so
# (the same sources with round 5's padded relayouts and natural-order Z row), three interleaved
# rounds of the C5 line (conforming path: kernel 7) and of the per-n_fft kernel-7 batches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-r06_swz_ab}
mkdir -p $O
for r in 1 2 3; do
  for v in product preswz; do
    if [ $v = preswz ]; then export THESIA_LIB=$PWD/multi-spectrogram-viewer_amd/lib/var/preswz.so; else unset THESIA_LIB; fi
    timeout -k 10 200 python bench.py --workload c5 --no-cpu-baseline > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err || { tail -5 $O/c5_${v}_$r.err; exit 1; }
    timeout -k 10 120 python scripts/r06/stftq_var_run.py > $O/k7_${v}_$r.txt 2>&1 || { tail -5 $O/k7_${v}_$r.txt; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/c5_${v}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$r $v c5 step %.3f spec %.3f display %.3f' % (d['ms_per_step'], r['overlapped_ms'], d['roofline_display']['display_ms']), [round(b['kernel_ms'],3) for b in r['per_batch']])"
    tr '\n' ' ' < $O/k7_${v}_$r.txt; echo
  done
done
