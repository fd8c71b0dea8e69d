#!/bin/bash
# C5 spectrogram kernels after the compile-time kinds: one SQ pass (issue vs waits) over the
# stft3 launches of the C5 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
R=$PWD
O=$R/gpurun_out/${1:-r05_c5spec2}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-include-regex "stft3" -d $O/pmc -o p --output-format csv -- python3 $R/bench.py --workload c5 --steps 3 --warmup 1 --no-exact > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -3 $O/pmc.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(o + "/pmc/p_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"].split("(")[0], r["Counter_Name"])
        tot[k] += float(r["Counter_Value"]); n[k] += 1
for k in sorted(tot):
    print(k[0], k[1], "%.4g" % (tot[k] / n[k]), n[k])
PY
