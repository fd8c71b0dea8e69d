#!/bin/bash
# LDS bank conflicts of stftq by variant (experiment library): 0 product, 16 lane-exchange swaps
# instead of the LDS relayout, 4 the FFT and the Z row alone. One rocprofv3 pass per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/${1:-r06_stftq_var}
mkdir -p $O
export TMPDIR=/tmp THESIA_LIB=$R/multi-spectrogram-viewer_amd/lib/libthesia_exp.so
cd /tmp
for v in 0 16 4; do
  THESIA_STFT_VARIANT=$v timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --kernel-include-regex "stftq" -d $O/v$v -o p --output-format csv -- python3 $R/scripts/r06/stftq_var_run.py > $O/v$v.log 2>&1 || { echo "variant $v failed"; tail -3 $O/v$v.log; exit 1; }
  grep "^[0-9]" $O/v$v.log
done
python3 - $O <<'PY'
import csv, glob, sys, collections, os
o = sys.argv[1]
for v in ("0", "16", "4"):
    tot = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob(f"{o}/v{v}/p_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = (r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])
            tot[k] += float(r["Counter_Value"]); n[k] += 1
    for k in sorted(tot):
        print("var", v, k[0], k[1], "%.4g" % (tot[k] / n[k]))
PY
