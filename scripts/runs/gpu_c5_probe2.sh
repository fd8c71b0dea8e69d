#!/bin/bash
# n_fft 1024 amp-dB launches of C5-batch size (250 tracks) vs larger ones, block counts varied
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/c5probe2; mkdir -p $O
for cfg in "250 24000" "1000 24000" "250 48000" "250 8000"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --workload c4 --tracks $1 --seconds 10 --sr $2 --channels 1 --input s16 --n-fft 1024 --hop 256 --output amp_db --no-cpu-baseline --no-e2e --no-rfft-roofline --no-c1 --steps 5 --warmup 1 --max-blocks 0,1024,512,256,128 > $O/b_$1_$2.log 2>&1 || exit $?
  python3 -c "
import json
L=open('$O/b_$1_$2.log').read().strip().splitlines()
d=json.loads(L[-1]); f=d['config']['frames_per_gpu']
mb=[json.loads(x) for x in L if 'max_blocks_ms' in x][0]['max_blocks_ms']
print('$cfg', f, {k: (round(v['median'],3), round(f/v['median']/1e6,3)) for k,v in mb.items()})"
done
