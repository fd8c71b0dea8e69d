set -o pipefail
O=gpurun_out/r05_scal; mkdir -p $O
F="--no-cpu-baseline --no-exact --no-e2e --no-rfft-roofline --no-c1 --output amp_db --channels 1 --seconds 10 --steps 20"
for t in 150 1000; do for k in 3 5; do
  timeout -k 10 200 python bench.py $F --tracks $t --kernel $k > $O/t${t}_k$k.json 2> $O/t${t}_k$k.err || exit 1
done; done
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['value'])"; done
