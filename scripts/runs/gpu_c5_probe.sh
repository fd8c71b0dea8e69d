set -o pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/c5probe; mkdir -p $O
timeout -k 10 200 python3 bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline > $O/c5.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('$O/c5.log').read().strip().splitlines()[-1]); print(d['roofline']['per_batch'])"
for cfg in "24000 256 64" "24000 512 128" "24000 1024 256" "24000 2048 512"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --workload c4 --tracks 1000 --seconds 10 --sr $1 --channels 1 --input s16 --n-fft $2 --hop $3 --output amp_db --no-cpu-baseline --no-e2e --no-rfft-roofline --no-c1 --steps 5 --warmup 1 > $O/big_$2.log 2>&1 || exit $?
  python3 -c "import json; d=json.loads(open('$O/big_$2.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['config']['frames_per_gpu'], round(r['kernel_ms'],3), round(r['frac'],3), r['kernel'][:40])"
done
