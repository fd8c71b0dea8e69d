#!/bin/bash
# stftr_kernel (C4, bit-exact mel-dB) SQ counters per launch for the ablation variants given
# (experiment library; 0 = the shipped kernel, 4 = the FFT alone). Two SQ passes per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/${1:-r05_pmc}
shift
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for v in "${@:-0}"; do
  i=0
  for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"; do
    THESIA_LIB=$R/multi-spectrogram-viewer_amd/lib/libthesia_exp.so THESIA_STFT_VARIANT=$v \
      timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "stftr" -d $O/v${v}_$i -o p --output-format csv -- \
      python3 $R/bench.py --kernel 7 --steps 3 --warmup 1 --no-cpu-baseline --no-c1 --no-e2e --no-rfft-roofline \
      > $O/v${v}_$i.log 2>&1 || { echo "variant $v pass $i failed"; tail -3 $O/v${v}_$i.log; exit 1; }
    i=$((i+1))
  done
done
python3 - $O <<'PY'
import csv, glob, sys, collections, os
o = sys.argv[1]
for d in sorted({os.path.basename(p).split("_")[0] for p in glob.glob(o + "/v*_*") if os.path.isdir(p)}):
    tot = collections.defaultdict(float); n = collections.Counter()
    for f in sorted(glob.glob(f"{o}/{d}_*/p_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(d, {k: "%.4g" % (tot[k] / n[k]) for k in sorted(tot)})
PY
