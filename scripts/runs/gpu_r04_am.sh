#!/bin/bash
# Round 4: ds_write_addtid_b32 address probe, then one LDS PMC pass over the product stft5 (C4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
O=$R/gpurun_out/${1:-r04_am}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 scripts/probes/addtid_probe > $O/probe.txt 2>&1 || { cat $O/probe.txt; exit 1; }
cut -c1-600 $O/probe.txt
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "stft5" -d $O/pmc -o p --output-format csv -- python3 $R/bench.py --kernel 5 --steps 3 --warmup 1 --no-cpu-baseline --no-c1 --no-rfft-roofline > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -3 $O/pmc.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in sorted(glob.glob(o + "/pmc/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"][:48], r["Counter_Name"])
        tot[k] += float(r["Counter_Value"]); n[k] += 1
for k in sorted(tot):
    print(k[0], k[1], "%.4g" % (tot[k] / n[k]), "per launch over", n[k])
PY
echo done
