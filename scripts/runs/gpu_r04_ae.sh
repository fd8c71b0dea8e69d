#!/bin/bash
# Round 4: counters of the stft5 phase-ring variant (experiment build, THESIA_STFT_VARIANT=1) vs the
# shipped kernel (0) on the C4 shard: SQ_INSTS_VALU / LDS / SALU, waits; and their times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_ae}
mkdir -p $O
export TMPDIR=/tmp THESIA_LIB=$R/multi-spectrogram-viewer_amd/lib/libthesia_exp.so
cd /tmp
for v in 0 1; do
  THESIA_STFT_VARIANT=$v timeout -k 10 300 python3 $R/bench.py --steps 10 --warmup 2 > $O/c4_v$v.json 2> $O/c4_v$v.err || { tail -5 $O/c4_v$v.err; exit 1; }
  tail -1 $O/c4_v$v.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('variant $v', round(d['ms_per_step'],3))"
  THESIA_STFT_VARIANT=$v timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex "stft5" -d $O/pmc_v$v -o p --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 > $O/pmc_v$v.log 2>&1 || { echo "pmc $v failed"; tail -3 $O/pmc_v$v.log; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
for v in (0, 1):
    tot = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f"{o}/pmc_v{v}/p_counter_collection.csv")):
        if "stft5_kernel<2, 2, 0" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print("variant", v, {k: "%.4g" % (tot[k] / n[k]) for k in sorted(tot)})
PY
echo done
